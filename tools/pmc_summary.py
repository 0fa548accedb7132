"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh for render_kernel into one JSON
(profiles/<round>_pmc.json).  HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section:
FETCH_SIZE is in KiB and counts half of the bytes of wide streaming reads on gfx950 (x2),
WRITE_SIZE is exact (KiB).  Usage: python tools/pmc_summary.py gpurun_out OUT.json [label] [precision]"""
import csv
import json
import os
import sys


PREC_TEMPLATE = {"fp32": 0, "bf16x3": 1, "bf16x6": 2, "fp16x3": 3, "fp16x4": 4}


def rows(path, kernel="render_kernel"):
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r["Kernel_Name"]:
                d = out.setdefault(r["Dispatch_Id"], {"ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def per_call(d, launches):
    """every counter summed over the LAST render_rays call's `launches` render_kernel dispatches (by dispatch id):
    the timed step's.  The passes run `bench.py --no-tally`, so the run's only dispatches of this instance are its
    warmup and timed steps; round 5's summary averaged in the untimed count_mfma tally call as well (VERDICT r5,
    What's weak 3: 596 MB instead of the timed call's 459 MB)."""
    ids = sorted(d, key=int)
    if len(ids) % launches:
        raise SystemExit(f"{len(ids)} dispatches is not a whole number of {launches}-launch calls")
    tot = {}
    for i in ids[-launches:]:
        for k, x in d[i].items():
            tot[k] = tot.get(k, 0.0) + x
    return tot, len(ids) // launches


def main():
    base, out_path = sys.argv[1], sys.argv[2]
    label = sys.argv[3] if len(sys.argv) > 3 else ""
    prec = sys.argv[4] if len(sys.argv) > 4 else "fp32"
    launches = int(sys.argv[5]) if len(sys.argv) > 5 else 2  # coarse + fine launch per render_rays call
    kern = f"render_kernel<256, 7, {PREC_TEMPLATE[prec]}>"  # this precision's instance only
    f, calls = per_call(rows(os.path.join(base, "pmc_fetch", "run_counter_collection.csv"), kern), launches)
    w, _ = per_call(rows(os.path.join(base, "pmc_write", "run_counter_collection.csv"), kern), launches)
    s, _ = per_call(rows(os.path.join(base, "pmc_sq", "run_counter_collection.csv"), kern), launches)
    hbm = 2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024
    clock = s["GRBM_GUI_ACTIVE"] / 8 / (s["ns"] * 1e-9) / 1e9
    busy = s["SQ_INSTS_MFMA"] / 1024 * 64 / (s["ns"] * 1e-9 * clock * 1e9)
    res = {
        "kernel": kern + " " + label,
        "precision": prec,
        "source": "rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES "
                  "GRBM_GUI_ACTIVE (separate passes) --kernel-trace -- python3 bench.py --steps 1 --warmup 1 --no-cpu "
                  "--no-tally --precision <precision> (tools/gpu_pmc.sh)",
        "unit": f"per render_rays call of one config-3 frame = {launches} render_kernel launches (coarse, fine) of the "
                f"timed step (the last of the {calls} calls each pass made: warmup + timed, no MFMA-tally call)",
        "FETCH_SIZE_KB_per_launch": f["FETCH_SIZE"],
        "WRITE_SIZE_KB_per_launch": w["WRITE_SIZE"],
        "render_kernel_hbm_bytes_per_launch": int(hbm),
        "hbm_bytes_note": "2 x FETCH_SIZE x 1024 (gfx950 half-count correction) + WRITE_SIZE x 1024, per call",
        "SQ_INSTS_MFMA": s["SQ_INSTS_MFMA"],
        "SQ_INSTS_VALU": s["SQ_INSTS_VALU"],
        "SQ_WAVES": s["SQ_WAVES"],
        "GRBM_GUI_ACTIVE": s["GRBM_GUI_ACTIVE"],
        "kernel_ns": s["ns"],
        "effective_clock_GHz": round(clock, 4),
        "mfma_pipe_busy_frac": round(busy, 4) if prec == "fp32" else None,
        "mfma_busy_note": "fp32 only: SQ_INSTS_MFMA / 1024 SIMDs x 64 cycles (v_mfma_f32_32x32x2_f32) / (time x clock)",
        "valu_per_mfma": round(s["SQ_INSTS_VALU"] / s["SQ_INSTS_MFMA"], 3),
    }
    json.dump(res, open(out_path, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
