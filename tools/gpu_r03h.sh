#!/bin/bash
# Round-3 session h: the whole GPU suite (cutoff_bones fixtures included), then identity + speed of the
# product build against tools/ab/lib_vcull.so (the same kernels before --cutoff_bones).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03h}
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
B=vcull BPRECS="bf16x6 fp32" bash tools/gpu_ab_out.sh || exit 1
exit $rc
