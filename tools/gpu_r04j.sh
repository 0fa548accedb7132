#!/bin/bash
# round 4: training GEMMs — forward GEMM time against K (slope = k-loop, intercept = per-tile prologue /
# epilogue), the 64-row tile variant (4 workgroups per CU) for correctness and speed, training-step A/B;
# then the bf16x6 scheduling A/B of tools/gpu_r04e.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r04j_gemm.txt
for p in 3 6; do
  for k in 64 128 256 512 1024; do
    timeout -k 10 120 python tools/gemm_bench.py --prec $p --k $k --cases forward || exit 1
  done
done 2>&1 | tee $O
echo "== bm64 correctness" | tee -a $O
ANERF_LIB_PATH=$PWD/tools/ab/lib_gbm64.so timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -3 | tee -a $O
LIBS="bm128 bm64" CASES=forward,input_grad bash tools/gpu_gemm_libs.sh 2>&1 | tee -a $O || exit 1
for r in 1 2; do
  for l in bm128 bm64; do
    echo "== train $l" | tee -a $O
    ANERF_LIB_PATH=$PWD/tools/ab/lib_g$l.so timeout -k 10 300 python tools/train_bench.py --steps 10 2>&1 | tail -1 | tee -a $O || exit 1
  done
done
echo "== fp16x4 render A/B: lock step (f4s), + persistent XCD-banded queues (f4p), lock step without block sort (f4b)"
LIBS="f4s:fp16x4 f4p:fp16x4 f4b:fp16x4" bash tools/gpu_ab3.sh 2>&1 | tee gpurun_out/r04j_ab_render.txt || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_f4s.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_f4s.npz fp16x4 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_f4p.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_f4p.npz fp16x4 || exit 1
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/ab_out_f4s.npz"), np.load("gpurun_out/ab_out_f4p.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("f4p vs f4s:", "bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
ANERF_LIB_PATH=$PWD/tools/ab/libanerf_hip_stamps.so ANERF_PRECISION=fp16x4 timeout -k 10 300 python tools/stamps.py \
    > gpurun_out/r04j_stamps_fp16x4.txt 2>&1 || exit 1
cat gpurun_out/r04j_stamps_fp16x4.txt
