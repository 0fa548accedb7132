#!/bin/bash
# A/B/C of experiment builds (tools/build_ab.sh) on one box: alternating bench runs, config 3.
#   LIBS="base ntv ntvg" PREC=bf16x6 bash tools/gpu_ab3.sh      (an entry NAME:PREC overrides PREC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for e in ${LIBS:-base}; do
    l=${e%%:*}; p=${PREC:-bf16x6}; [ "$e" != "$l" ] && p=${e#*:}
    v=$(ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 300 python bench.py --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision $p 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "$e $v"
  done
done
