#!/bin/bash
# round 5: hidden-layer boundary (tail max) -- layer probe old/new, then A/B base / enc16 / tail (fp16x4)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05c
{ echo "== h4_probe_4 (round 4 layer)"; timeout -k 10 120 ./tools/probe/h4_probe_4 || exit 1
  echo "== h4_probe_4t (round 5: tail max)"; timeout -k 10 120 ./tools/probe/h4_probe_4t || exit 1; } | tee gpurun_out/${TAG}_probe.txt
LIBS="base enc16 tail" PREC=fp16x4 bash tools/gpu_ab3.sh | tee gpurun_out/${TAG}_ab.txt
