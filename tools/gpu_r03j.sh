#!/bin/bash
# kernel stats of the training step, fused forward vs layer-by-layer GEMMs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in fused gemm; do
  ANERF_TRAIN_FWD=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof_$m -o run --output-format csv -- python3 tools/train_bench.py --steps 10 --warmup 2 > gpurun_out/tprof_$m.log 2>&1 || { tail -5 gpurun_out/tprof_$m.log; exit 1; }
  echo "== $m"; head -14 gpurun_out/tprof_$m/run_kernel_stats.csv | cut -d, -f1-4
done
