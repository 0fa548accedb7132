#!/bin/bash
# round 5: the staged-encoder suite (+ querypts) and the training goldens on the product build, then the whole GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05q
timeout -k 10 300 python -u -m pytest tests/test_gpu_staged.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_staged.log 2>&1 || { tail -30 gpurun_out/${TAG}_staged.log; exit 1; }
tail -2 gpurun_out/${TAG}_staged.log
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -15
exit $rc
