#!/bin/bash
# kernel stats of the training step, relu' masks as bits vs fp32 activations
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 1 0; do
  ANERF_TRAIN_BITS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tprofb_$b -o run --output-format csv -- python3 tools/train_bench.py --steps 10 --warmup 2 > gpurun_out/tprofb_$b.log 2>&1 || { tail -5 gpurun_out/tprofb_$b.log; exit 1; }
done
