#!/bin/bash
# round 6: the fused hidden-layer backward -- MLP / train tests, then training A/B (fused vs two GEMMs, pose chain on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06b
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "backward_hidden" > gpurun_out/${TAG}_pytest_dgw.log 2>&1; rc=$?
tail -5 gpurun_out/${TAG}_pytest_dgw.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py tests/test_kinematics.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_train.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest_train.log
[ $rc -eq 0 ] || exit $rc
for v in fused two fused two; do
  f=""; [ $v = two ] && f="--no-fused-backward"
  timeout -k 10 200 python tools/train_bench.py --steps 20 $f 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_train_ab.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_tprof -o run --output-format csv -- python3 tools/train_bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_tprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_tprof.log; exit 1; }
