#!/bin/bash
# round 5: the GPU suite on the ABI-15 product build (staged encoders, generic training multires, world views)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05l
timeout -k 10 300 python -u -m pytest tests/test_gpu_staged.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_staged.log 2>&1; rc=$?
tail -15 gpurun_out/${TAG}_staged.log
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc2=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
exit $((rc | rc2))
