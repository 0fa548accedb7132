#!/bin/bash
# weight gradients on the side stream vs the caller's stream, with the view-window layout (A/B, interleaved)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r05zs
for i in 1 2; do
  for v in "" "--no-wgrad-overlap"; do
    timeout -k 10 200 python tools/train_bench.py --steps 20 $v 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${v:-overlap}', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_ab.txt || exit 1
  done
done
