#!/bin/bash
# A/B of experiment builds (tools/build_ab.sh) on the density path: alternating tools/density_bench.py
# runs (256^3 grid, config-3 fine net).   LIBS="a b" PREC=bf16x6 bash tools/gpu_ab_density.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for l in ${LIBS:-base}; do
    v=$(ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 200 python tools/density_bench.py 255 ${PREC:-bf16x6} 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['ms'], d['finite'])") || exit 1
    echo "$l $v"
  done
done
