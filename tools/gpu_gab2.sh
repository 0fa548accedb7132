#!/bin/bash
# weight-gradient workgroups per launch (ANERF_WGRAD_WG): training step A/B across experiment builds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2; do
  for v in base bm64 bd2; do
    ANERF_LIB_PATH=$PWD/tools/ab/lib_g$v.so timeout -k 10 200 python tools/train_bench.py --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/gab2.txt || exit 1
  done
done
