"""Summarise tools/gpu_r04l.sh's SQ counter passes per kernel: the share of wave cycles parked at
s_waitcnt / barriers (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY; LDS issue stalls a sub-bucket),
issuing (SQ_ACTIVE_INST_ANY), and the MFMA pipe's busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
GRBM_GUI_ACTIVE x 4 SIMDs per CU, MI355X_MICROARCH.md units: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* in
quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES in cycles, summed over the chip's 256 CUs; GRBM_GUI_ACTIVE per
XCD).  Usage: python tools/pmc_waves.py DIR ..."""
import csv
import re
import glob
import os
import sys


def kernels(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = {}
    for r in csv.DictReader(open(f[0])):
        k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
        k = re.sub(r"^void ", "", k).split("(")[0][:60]
        e = out.setdefault(k, {"n": set(), "ns": 0})
        if r["Dispatch_Id"] not in e["n"]:
            e["n"].add(r["Dispatch_Id"])
            e["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


for d in sys.argv[1:]:
    print(f"== {d}")
    for k, e in sorted(kernels(d).items(), key=lambda kv: -kv[1]["ns"]):
        if "SQ_WAVE_CYCLES" not in e or e["SQ_WAVE_CYCLES"] == 0 or e["ns"] < 20000:
            continue
        wc = e["SQ_WAVE_CYCLES"]
        grbm = e.get("GRBM_GUI_ACTIVE", 0.0) / 8  # per XCD -> per GPU cycles
        mf = e.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (grbm * 1024) if grbm else float("nan")
        print(f"{k:60s} calls {len(e['n']):4d} avg_us {e['ns'] / len(e['n']) / 1e3:9.1f}  "
              f"waits {e.get('SQ_WAIT_ANY', 0) / wc:5.2f}  issue-stall {e.get('SQ_WAIT_INST_ANY', 0) / wc:5.2f} "
              f"(lds {e.get('SQ_WAIT_INST_LDS', 0) / wc:4.2f})  active {e.get('SQ_ACTIVE_INST_ANY', 0) / wc:5.2f}  "
              f"mfma-busy/SIMD {mf:5.2f}  waves/SIMD {wc / (grbm / 4 * 1024) if grbm else float('nan'):4.2f}")
