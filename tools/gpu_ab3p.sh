#!/bin/bash
# A/B of experiment builds like tools/gpu_ab3.sh, also printing each run's parity leg (max |gpu - oracle| on
# 20,000 rays of the frame: rgb, disp, acc)
#   LIBS="a b:fp16x3" PREC=fp16x4 bash tools/gpu_ab3p.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for e in ${LIBS:-base}; do
    l=${e%%:*}; p=${PREC:-fp16x4}; [ "$e" != "$l" ] && p=${e#*:}
    v=$(ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 300 python bench.py --cpu-rays 2000 --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision $p 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernel_ms'], d['parity']['max_abs_err'])") || exit 1
    echo "$e $v"
  done
done
