#!/bin/bash
# GEMM numerics tests, microbenchmark, and the diagnostic timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-gt}
bash tools/gpu_gemm_quick.sh || exit 1
ANERF_GEMM_STAMPS=1 timeout -k 10 60 python tools/gemm_timeline.py | tee gpurun_out/${TAG}_timeline.txt
