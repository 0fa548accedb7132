#!/bin/bash
# persistent forward timing probes (wrong results): micro (forward_persistent, M = 163,840) per probe build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
for r in 1 2; do for p in 0 1 2 3 4; do
  L=""; [ $p != 0 ] && L=tools/ab/lib_gfwp$p.so
  ANERF_LIB_PATH=$L timeout -k 10 120 python tools/gemm_bench.py --prec 6 --cases forward_persistent > $O/p$p.json 2>> $O/err || exit 1
  python -c "import json;d=json.load(open('$O/p$p.json'));print('probe $p', d['us'])" | tee -a $O/probes.txt
done; done
