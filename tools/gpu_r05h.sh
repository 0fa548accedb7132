#!/bin/bash
# round 5: product build (enc16 + fma_mix split + lead-group pin + 16-B z hand-off): GPU tests, then the
# write accounting passes (tools/gpu_r05g.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05h
timeout -k 10 900 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash tools/gpu_r05g.sh
timeout -k 10 60 ./tools/probe/mfma_f8_probe | tee gpurun_out/r05h_f8probe.txt
