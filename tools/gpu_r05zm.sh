#!/bin/bash
# torch Adam fused vs foreach in the training step (A/B, interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r05zm
for i in 1 2; do
  for v in fused foreach; do
    timeout -k 10 200 python tools/train_bench.py --steps 20 --adam $v 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_adam_ab.txt || exit 1
  done
done
