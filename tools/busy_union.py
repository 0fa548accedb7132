"""GPU busy time per step from a rocprofv3 --kernel-trace CSV: the union of the kernels' [start, end) intervals
(two streams overlap) against the wall span, and the idle gaps longer than a threshold.
usage: python tools/busy_union.py <kernel_trace.csv> [--from-kernel NAME] [--gap-us 20]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--gap-us", type=float, default=20.0)
ap.add_argument("--skip-first", type=int, default=0, help="ignore this many leading kernels (warmup)")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.csv)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)[a.skip_first:]
busy, cur_s, cur_e = 0, iv[0][0], iv[0][1]
gaps = []
prev_name = iv[0][2]
for s, e, nm in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        if (s - cur_e) / 1e3 >= a.gap_us:
            gaps.append(((s - cur_e) / 1e3, prev_name[:60], nm[:60]))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev_name = nm if e >= cur_e else prev_name
busy += cur_e - cur_s
span = iv[-1][1] - iv[0][0]
print(f"kernels {len(iv)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  idle {(span - busy) / 1e6:.3f} ms "
      f"({100 * (span - busy) / span:.1f} %)")
print(f"gaps >= {a.gap_us} us: {len(gaps)}, total {sum(g[0] for g in gaps) / 1e3:.3f} ms")
for g in sorted(gaps, reverse=True)[:30]:
    print(f"  {g[0]:9.1f} us  after {g[1]}  before {g[2]}")
