#!/bin/bash
# round 4: full GPU tests of the product build (block sort, u-features unroll, multires 1-10 / views 0-4,
# GEMM staging interleave), then the A/B session (tools/gpu_r04e.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/r04f_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r04f_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
bash tools/gpu_r04e.sh || exit 1
exit $rc
