#!/bin/bash
# Round-3 session n: windowed part as bf16x6 (v_part_x6): render parity tests, output diff against the
# previous build (tools/ab/lib_$B.so), then alternating bench runs A (in-tree) / B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03n}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | tail -12
[ $rc -eq 0 ] || exit $rc
B=${B:-head} PRECS="bf16x6 fp16x3" BPRECS="bf16x6 fp16x3" timeout -k 10 900 bash tools/gpu_ab_out.sh
