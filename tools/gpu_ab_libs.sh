#!/bin/bash
# A/B of two builds on one box: alternate bench runs of the in-tree library and tools/libanerf_hip_prev.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2 3; do
  for lib in a-nerf_amd/libanerf_hip.so tools/libanerf_hip_prev.so; do
    v=$(ANERF_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu --precision ${PREC:-bf16x6} 2>/dev/null | python -c "import json,sys;d=json.load(sys.stdin);print(d['value'], d['roofline']['kernel_ms'])") || exit 1
    echo "$lib $v"
  done
done
