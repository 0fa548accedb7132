#!/bin/bash
# round 5: timing bound of the view-direction part (novdir: the part removed, wrong outputs, timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2 3; do for l in base novdir; do
  v=$(ANERF_LIB_PATH=$PWD/tools/ab/lib_$l.so timeout -k 10 300 python bench.py --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision fp16x4 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernel_ms'])") || exit 1
  echo "$l $v"
done; done | tee gpurun_out/r05w_ab.txt
