#!/bin/bash
# round 4: the bf16x3 NT GEMM with 64-column k-steps (half the barriers, twice the A bytes in flight):
# correctness (test_gpu_mlp), GEMM microbench and training-step A/B against 32-column steps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r04w_gemm_sk64.txt
for l in sk64 sk64b2; do
  echo "== $l correctness" | tee -a $O
  ANERF_LIB_PATH=$PWD/tools/ab/lib_g$l.so timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -2 | tee -a $O
done
LIBS="sk32 sk64 sk64b2" PRECS=3 CASES=forward,input_grad bash tools/gpu_gemm_libs.sh 2>&1 | grep -v amdgpu.ids | tee -a $O || exit 1
for r in 1 2; do
  for l in sk32 sk64 sk64b2; do
    echo "== train $l" | tee -a $O
    ANERF_LIB_PATH=$PWD/tools/ab/lib_g$l.so timeout -k 10 300 python tools/train_bench.py --steps 10 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])" | tee -a $O || exit 1
  done
done
