#!/bin/bash
# round 4: is the NT GEMM's k-loop waiting on its A loads?  The same kernel with every tile reading
# the first 128 rows (L2-hot A, wrong results, timing only) against the product build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="cur probeA" CASES=forward,input_grad bash tools/gpu_gemm_libs.sh 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04t_gemm_probeA.txt || exit 1
