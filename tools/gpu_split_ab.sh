#!/bin/bash
# Same-box A/B of the batched weight split: the training bench alternating batched / per-weight splits.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-sab}
for r in 1 2; do
  timeout -k 10 200 python tools/train_bench.py | tee -a gpurun_out/${TAG}.jsonl || exit 1
  timeout -k 10 200 python tools/train_bench.py --split-single | tee -a gpurun_out/${TAG}_single.jsonl || exit 1
done
echo ok
