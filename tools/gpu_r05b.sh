#!/bin/bash
# round 5: fp16 encoder-fed parts (enc16) -- GPU tests, then A/B against the round-4 kernel (tools/ab/lib_base.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05b
timeout -k 10 900 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
LIBS="base enc16 base:fp16x3 enc16:fp16x3" PREC=fp16x4 bash tools/gpu_ab3.sh | tee gpurun_out/${TAG}_ab.txt
