#!/bin/bash
# round 5: the composite's wave index as a scalar (cw1) vs the product (base): per-dispatch WRITE_SIZE and the render A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05o
for l in base cw1; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${T}_w_$l -o run --output-format csv -- python3 tools/write_probe.py > gpurun_out/${T}_w_$l.log 2>&1 || { tail -20 gpurun_out/${T}_w_$l.log; exit 1; }
done
LIBS="base cw1" PREC=fp16x4 bash tools/gpu_ab3p.sh | tee gpurun_out/${T}_ab.txt
