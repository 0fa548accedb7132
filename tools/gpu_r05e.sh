#!/bin/bash
# round 5: VALU pin in the fp16 layers' lead groups (ANERF_H3_LEAD_IL 2 / 4 / 6), fp16x4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="mix lead4 lead6" PREC=fp16x4 bash tools/gpu_ab3.sh | tee gpurun_out/r05e_ab.txt
