#!/bin/bash
# Bit-identity and speed of an experiment build (tools/ab/lib_$B.so) against the in-tree library:
# the config-3 frame's outputs from both (tools/ab_outputs.py) compared exactly, then the A/B bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_A.npz ${PRECS:-bf16x6 fp16x3 fp32} || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_$B.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_B.npz ${PRECS:-bf16x6 fp16x3 fp32} || exit 1
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/ab_out_A.npz"), np.load("gpurun_out/ab_out_B.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("bit-identical" if not bad else f"DIFFER: {bad[:8]} max {max(float(np.nanmax(np.abs(a[k] - b[k]))) for k in bad):.3e}")
PY
for r in 1 2 3; do
  for l in A B; do
    lib=$PWD/a-nerf_amd/libanerf_hip.so; [ $l = B ] && lib=$PWD/tools/ab/lib_$B.so
    for p in ${BPRECS:-bf16x6 fp16x3}; do
      v=$(ANERF_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu --no-tau20 --no-train --also "" --precision $p 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac_executed'])") || exit 1
      echo "$l $p $v"
    done
  done
done
