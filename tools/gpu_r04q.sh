#!/bin/bash
# round 4: fp16 layers scaled from a bound on their input (no drain at the layer boundary): probe,
# render A/B against the exact-max build, parity against the oracle on bench.py's 20 k rays
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="f4p:fp16x4 f4bd:fp16x4 f4p:fp16x3 f4bd:fp16x3" bash tools/gpu_ab3.sh 2>&1 | tee gpurun_out/r04q_ab.txt || exit 1
for l in f4p f4bd; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 400 python bench.py --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision fp16x4 > gpurun_out/r04q_parity_$l.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04q_parity_$l.json')); print('$l', d['value'], json.dumps(d['parity']['max_abs_err']), d['parity']['near_empty_disp_max_abs_err'])" | tee -a gpurun_out/r04q_ab.txt
done
