#!/bin/bash
# round 4: packed-fp32 splits (ANERF_SPLIT_PK) A/B in fp16x4, bf16x6, fp16x3; parity of the new fp16 split
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="pk0:fp16x4 pk1:fp16x4 pk0:bf16x6 pk1:bf16x6" bash tools/gpu_ab3.sh 2>&1 | tee gpurun_out/r04r_ab.txt || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_pk0.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_A.npz bf16x6 || exit 1
ANERF_LIB_PATH=$PWD/tools/ab/lib_pk1.so timeout -k 10 300 python tools/ab_outputs.py gpurun_out/ab_out_B.npz bf16x6 || exit 1
python - <<'PY' | tee -a gpurun_out/r04r_ab.txt
import numpy as np
a, b = np.load("gpurun_out/ab_out_A.npz"), np.load("gpurun_out/ab_out_B.npz")
bad = [k for k in a.files if not np.array_equal(a[k], b[k], equal_nan=True)]
print("bf16x6 pk1 vs pk0:", "bit-identical" if not bad else f"DIFFER: {bad[:8]}")
PY
for l in pk0 pk1; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 400 python bench.py --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision fp16x4 > gpurun_out/r04r_parity_$l.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04r_parity_$l.json')); print('$l fp16x4', d['value'], json.dumps(d['parity']['max_abs_err']), d['parity']['near_empty_disp_max_abs_err'])" | tee -a gpurun_out/r04r_ab.txt
done
