#!/bin/bash
# round 4: fp16x4 (four fp16 products) against bf16x6, with and without the hidden-layer lock step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="cur:bf16x6 f4:fp16x4 f4s:fp16x4 f4:fp16x3" bash tools/gpu_ab3.sh | tee gpurun_out/r04h_ab_f4.txt || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_f4s.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_f4s.npz fp16x4 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_f4.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_f4.npz fp16x4 || exit 1
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/ab_out_f4.npz"), np.load("gpurun_out/ab_out_f4s.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("f4s vs f4:", "bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
