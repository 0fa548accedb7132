#!/bin/bash
# rocprofv3 kernel stats of the final round-4 bench (headline fp16x4 only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04zd -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" > gpurun_out/r04zd_prof.log 2>&1 || { tail -20 gpurun_out/r04zd_prof.log; exit 1; }
f=$(find gpurun_out/prof_r04zd -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/r04zd_kernel_stats.csv
rm -rf gpurun_out/prof_r04zd
tail -1 gpurun_out/r04zd_prof.log | cut -c1-300
python3 - <<'PY'
import csv
rows = sorted(csv.DictReader(open("gpurun_out/r04zd_kernel_stats.csv")), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:6]:
    print(f'{float(r["AverageNs"])/1e6:9.3f} ms x {r["Calls"]:>4}  {r["Name"][:90]}')
PY
