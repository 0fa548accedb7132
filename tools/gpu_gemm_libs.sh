#!/bin/bash
# GEMM microbenchmark (forward, input gradient) over the libraries named in LIBS (tools/ab/lib_gNAME.so),
# alternating, on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for n in ${LIBS:-base}; do
    for p in ${PRECS:-6 3}; do
      echo "== $n prec $p"
      ANERF_LIB_PATH=$PWD/tools/ab/lib_g$n.so timeout -k 10 120 python tools/gemm_bench.py --prec $p --cases ${CASES:-forward,input_grad} || exit 1
    done
  done
done
