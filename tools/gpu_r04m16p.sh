#!/bin/bash
# per-kernel times of the training step, mixed vs mixed16 (rocprofv3 --kernel-trace --stats)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in mixed mixed16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04m16p_$m -o run --output-format csv -- \
      python3 tools/train_bench.py --mlp $m --steps 5 --warmup 1 > gpurun_out/r04m16p_$m.txt 2>&1 || { tail -20 gpurun_out/r04m16p_$m.txt; exit 1; }
done
for m in mixed mixed16; do
  f=$(find gpurun_out/r04m16p_$m -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/r04m16p_${m}_kernel_stats.csv
  echo "== $m $f"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:14]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
done
rm -rf gpurun_out/r04m16p_mixed gpurun_out/r04m16p_mixed16
