#!/bin/bash
# round 5: f8 probe (+ accumulator precision under the scaled fp8 MFMA); render A/B with parity on 2,000 rays:
# uf0 (product render), f8x1 (x1 w1 in e4m3), uf1 (fused layer-0 bone-direction pass), uf1f8 (both)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05k
timeout -k 10 60 ./tools/probe/mfma_f8_probe | tee gpurun_out/${TAG}_f8probe.txt || exit 1
LIBS="uf0 f8x1 uf1 uf1f8" PREC=fp16x4 bash tools/gpu_ab3p.sh | tee gpurun_out/${TAG}_ab.txt
