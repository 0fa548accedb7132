#!/bin/bash
# round 4: power probes (what the clock pays for in the x6 layer); block sort + u-features A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for n in 0 1 2 3; do timeout -k 10 120 tools/probe/power_probe_$n || exit 1; done 2>&1 | tee gpurun_out/r04e_power_probe.txt
ANERF_LIB_PATH=$PWD/tools/ab/lib_sort0.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_A.npz bf16x6 fp32 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_per1.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_B.npz bf16x6 fp32 || exit 1
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/ab_out_A.npz"), np.load("gpurun_out/ab_out_B.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("per1 vs sort0:", "bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
LIBS="sort0 cur per1 xb0 xb1" PREC=bf16x6 bash tools/gpu_ab3.sh || exit 1
echo "== GEMM interleave: correctness (test_gpu_mlp with lib_gil1), then A/B"
ANERF_LIB_PATH=$PWD/tools/ab/lib_gil1.so timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or nerf_forward" 2>&1 | tail -3
LIBS="il0 il1" bash tools/gpu_gemm_libs.sh 2>&1 | grep -E "==|forward|input_grad" | python -c "
import sys,json
cur=None
for l in sys.stdin:
    if l.startswith('=='): cur=l.strip(); continue
    d=json.loads(l); print(cur, d['case'], d['us'], d['TFLOPs_ref'])"
