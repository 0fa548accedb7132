#!/bin/bash
# round 4: block order by live joints (ANERF_BLOCK_SORT) — outputs bit-identical, A/B speed, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
ANERF_LIB_PATH=$PWD/tools/ab/lib_sort0.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_A.npz bf16x6 fp32 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_sort1.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_B.npz bf16x6 fp32 || exit 1
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/ab_out_A.npz"), np.load("gpurun_out/ab_out_B.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
LIBS="sort0 sort1" PREC=bf16x6 bash tools/gpu_ab3.sh || exit 1
ANERF_PRECISION=bf16x6 timeout -k 10 300 python tools/stamps.py 79.6 > gpurun_out/r04d_stamps_bf16x6.txt 2>&1 || { tail gpurun_out/r04d_stamps_bf16x6.txt; exit 1; }
cat gpurun_out/r04d_stamps_bf16x6.txt
