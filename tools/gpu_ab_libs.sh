#!/bin/bash
# A/B of two builds on one box: alternate bench runs of the in-tree library and ${LIB_B:-tools/ab/libanerf_hip_b.so}
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for lib in a-nerf_amd/libanerf_hip.so ${LIB_B:-tools/ab/libanerf_hip_b.so}; do
    v=$(ANERF_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --no-tau20 --also "" --precision ${PREC:-fp16x3} 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "$lib $v"
  done
done
