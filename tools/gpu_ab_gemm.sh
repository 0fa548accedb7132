#!/bin/bash
# A/B of the GEMM microbenchmark between the in-tree library and ${LIB_B:-tools/ab/libanerf_hip_b.so}, alternating, on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for lib in a-nerf_amd/libanerf_hip.so ${LIB_B:-tools/ab/libanerf_hip_b.so}; do
    echo "== $lib"
    ANERF_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/gemm_bench.py --prec ${PREC:-6} --cases ${CASES:-forward,input_grad,weight_grad} || exit 1
  done
done
