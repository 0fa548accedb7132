#!/bin/bash
# Training MLP GEMMs: numerics tests, training parity, then the training bench (+ kernel stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-mlp}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py -x -q -s -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python tools/train_bench.py > gpurun_out/${TAG}_train_bench.json 2> gpurun_out/${TAG}_train_bench.err || { tail -20 gpurun_out/${TAG}_train_bench.err; exit 1; }
cat gpurun_out/${TAG}_train_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*stats*"
