#!/bin/bash
# Training bench in the three MLP arithmetic modes, then kernel stats of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-t3}
for m in ${MODES:-mixed bf16x6 bf16x3 fp32}; do timeout -k 10 200 python tools/train_bench.py --mlp $m | tee -a gpurun_out/${TAG}_train.jsonl || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
echo ok
