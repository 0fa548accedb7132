#!/bin/bash
# round 5: (1) GPU tests of the product build (256-column training GEMM tiles, fp8 x1w1 off); (2) fp8 probe and
# render A/B uf0 (product) / f8x1 / uf1 (fused u part) with parity; (3) training GEMM A/B: 128- vs 256-column tiles (gemm_bench, train_bench)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05j
timeout -k 10 900 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 60 ./tools/probe/mfma_f8_probe | tee gpurun_out/${TAG}_f8probe.txt || exit 1
for r in 1 2; do for l in gcb1 gcb2; do
  echo "== $l gemm"; ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 200 python tools/gemm_bench.py --prec 3 --cases forward,input_grad || exit 1
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 200 python tools/gemm_bench.py --prec 6 --cases forward || exit 1
done; done 2>&1 | tee gpurun_out/${TAG}_gemm.txt
for r in 1 2; do for l in gcb1 gcb2; do
  echo "== $l train"; ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 300 python tools/train_bench.py || exit 1
done; done 2>&1 | tee gpurun_out/${TAG}_train.txt
LIBS="uf0 f8x1 uf1 uf1f8" PREC=fp16x4 bash tools/gpu_ab3p.sh | tee gpurun_out/${TAG}_ab.txt
