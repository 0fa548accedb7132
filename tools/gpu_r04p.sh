#!/bin/bash
# round 4: h3_scale as a tree + v_permlane32_swap: layer probe, render A/B (fp16x4, fp16x3), bit-identity
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in h4_probe_4 h4_probe_4t; do echo "== $b"; timeout -k 10 120 tools/probe/$b || exit 1; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04p_probe.txt
LIBS="f4p:fp16x4 f4t:fp16x4 f4p:fp16x3 f4t:fp16x3" bash tools/gpu_ab3.sh 2>&1 | tee gpurun_out/r04p_ab.txt || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_f4p.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_A.npz fp16x4 fp16x3 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_f4t.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_B.npz fp16x4 fp16x3 || exit 1
python - <<'PY' | tee -a gpurun_out/r04p_ab.txt
import numpy as np
a, b = np.load("gpurun_out/ab_out_A.npz"), np.load("gpurun_out/ab_out_B.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("f4t vs f4p:", "bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
