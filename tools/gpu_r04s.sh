#!/bin/bash
# round 4: hidden-layer barriers (ANERF_X6_BARRIERS 3 = before every hidden layer, 2 = layer 1 and the
# one after the skip layer, 1 = layer 1 only) in fp16x4 and bf16x6 with the persistent queues
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="xb3:fp16x4 xb2:fp16x4 xb1:fp16x4 xb3:bf16x6 xb2:bf16x6" bash tools/gpu_ab3.sh 2>&1 | tee gpurun_out/r04s_ab.txt || exit 1
