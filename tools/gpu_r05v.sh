#!/bin/bash
# round 5: schedule knobs re-measured on the final build (interior VALU pin 3, one load group, two barriers,
# blocks in ray order) against the product schedule
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="base il3 nlg1 xb2 bs0" PREC=fp16x4 bash tools/gpu_ab3p.sh | tee gpurun_out/r05v_ab.txt
