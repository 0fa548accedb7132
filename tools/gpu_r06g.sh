#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "backward_hidden" > gpurun_out/r06g_pytest_dgw.log 2>&1; rc=$?
tail -3 gpurun_out/r06g_pytest_dgw.log
[ $rc -eq 0 ] || exit $rc
LIBS="base bd2 p4" TAG=r06g bash tools/gpu_r06c.sh || exit 1
for v in fused two fused two; do
  f=""; [ $v = two ] && f="--no-fused-backward"
  timeout -k 10 200 python tools/train_bench.py --steps 20 $f 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06g_train_ab.txt || exit 1
done
