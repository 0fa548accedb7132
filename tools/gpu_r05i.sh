#!/bin/bash
# round 5: fp8 x1 w1 (ANERF_F8_X1W1) -- the f8f6f4 MFMA probe, then A/B f8x0 / f8x1 (fp16x4) with parity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probe/mfma_f8_probe | tee gpurun_out/r05i_f8probe.txt || exit 1
LIBS="f8x0 f8x1" PREC=fp16x4 bash tools/gpu_ab3p.sh | tee gpurun_out/r05i_ab.txt
