#!/bin/bash
# round 5: fp16 split by v_fma_mix_f32 -- layer probe (plain and phase stamps), then A/B enc16 / mix (fp16x4, fp16x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05d
{ for b in h4_probe_4 h4_probe_4mix h4_probe_4st h4_probe_4mixst; do echo "== $b"; timeout -k 10 120 ./tools/probe/$b || exit 1; done; } | tee gpurun_out/${TAG}_probe.txt
LIBS="enc16 mix enc16:fp16x3 mix:fp16x3" PREC=fp16x4 bash tools/gpu_ab3.sh | tee gpurun_out/${TAG}_ab.txt
