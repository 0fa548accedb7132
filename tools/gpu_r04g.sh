#!/bin/bash
# round 4: fp16 with the fourth product (x1 w1) — speed (A/B against fp16x3) and its error against the
# C oracle on bench.py's 20 k-ray parity sample, next to bf16x6's and fp16x3's on the same rays
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="h3 h4" PREC=fp16x3 bash tools/gpu_ab3.sh | tee gpurun_out/r04g_ab_h4.txt || exit 1
for l in h3 h4; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 400 python bench.py --no-tau20 --no-train --no-balance \
      --other-configs "" --also "" --precision fp16x3 > gpurun_out/r04g_parity_$l.json 2> gpurun_out/r04g_parity_$l.err || exit 1
done
ANERF_LIB_PATH=$PWD/tools/ab/lib_h3.so timeout -k 10 400 python bench.py --no-tau20 --no-train --no-balance \
    --other-configs "" --also "" --precision bf16x6 > gpurun_out/r04g_parity_x6.json 2> gpurun_out/r04g_parity_x6.err || exit 1
for f in h3 h4 x6; do
  python -c "import json,sys; d=json.load(open('gpurun_out/r04g_parity_$f.json')); print('$f', d['value'], json.dumps(d.get('parity')))"
done
