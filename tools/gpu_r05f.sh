#!/bin/bash
# round 5: (1) joints per iteration of the bone-direction feature pass (ANERF_UF_UNROLL 2 / 4 / 6) and the
# 16-B z hand-off (zv), fp16x4 A/B; (2) WRITE_SIZE of the render kernel with 4-B (lead4) and 16-B (zv)
# z hand-off stores; (3) the TCC counter list
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="lead4 uf2 uf4 uf6 zv" PREC=fp16x4 bash tools/gpu_ab3.sh | tee gpurun_out/r05f_ab.txt || exit 1
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/r05f_avail.txt 2>&1 || true
for l in lead4 zv; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/r05f_pmcw_$l -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision fp16x4 > gpurun_out/r05f_pmcw_$l.log 2>&1 || { tail -20 gpurun_out/r05f_pmcw_$l.log; exit 1; }
done
grep -o -E "TCC_[A-Za-z0-9_]*" gpurun_out/r05f_avail.txt | sort -u | tr '\n' ' '
