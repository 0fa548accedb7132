#!/bin/bash
# Round-3 session i: the fused training forward (anerf_mlp_forward): MLP + training GPU tests, then the
# training step fused vs layer-by-layer GEMM forward (ANERF_TRAIN_FWD=gemm), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03i}
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | tail -12
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for m in fused gemm; do
    v=$(ANERF_TRAIN_FWD=$m timeout -k 10 200 python tools/train_bench.py --steps 10 --warmup 2 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$m $v"
  done
done
