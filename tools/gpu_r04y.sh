#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="h3free:fp16x3 h3lock:fp16x3" bash tools/gpu_ab3.sh 2>&1 | tee gpurun_out/r04y_ab_h3lock.txt || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_h3free.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_A.npz fp16x3 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_h3lock.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_B.npz fp16x3 || exit 1
python - <<'PY' | tee -a gpurun_out/r04y_ab_h3lock.txt
import numpy as np
a, b = np.load("gpurun_out/ab_out_A.npz"), np.load("gpurun_out/ab_out_B.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("fp16x3 lock vs free:", "bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
