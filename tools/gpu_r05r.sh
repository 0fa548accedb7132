#!/bin/bash
# round 5: the feature pass skipping the view windows of view-dead joint pairs (wvs1) vs without (base), with parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="base wvs1 base:bf16x6 wvs1:bf16x6" PREC=fp16x4 bash tools/gpu_ab3p.sh | tee gpurun_out/r05r_ab.txt
