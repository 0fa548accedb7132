#!/bin/bash
# round 5: weight gradients on a second stream (overlapping the input gradients) vs the caller's stream; the
# training goldens and the MLP tests with the overlap on
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05s
for r in 1 2; do
  echo "== overlap"; timeout -k 10 300 python tools/train_bench.py || exit 1
  echo "== serial"; timeout -k 10 300 python tools/train_bench.py --no-wgrad-overlap || exit 1
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_train_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_mlp.py tests/test_gpu_staged.py -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest.log | tail -10
exit $rc
