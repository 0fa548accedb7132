#!/bin/bash
# persistent forward experiment builds: micro only.  usage: bash tools/gpu_fwmicro.sh <tag> <lib names...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O
for r in 1 2; do for v in base "$@"; do
  L=""; [ $v != base ] && L=tools/ab/lib_g$v.so
  ANERF_LIB_PATH=$L timeout -k 10 120 python tools/gemm_bench.py --prec 6 --cases forward_persistent > $O/m_$v.json 2>> $O/err || exit 1
  python -c "import json;d=json.load(open('$O/m_$v.json'));print('micro $v', d['us'])" | tee -a $O/ab.txt
done; done
