#!/bin/bash
# round 6: bounds on the training step -- skip the fused backward's slab reduce / the other weight gradients
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06n
mkdir -p $O
for rep in 1 2; do
for p in none no-hidden-reduce no-wgrad no-wgrad-no-reduce; do
  f=""; [ $p != none ] && f="--probe $p"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$p.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$p.json'));print('$p',d['value'],d['ms_per_step'],d['host_issue_ms_per_step'])"
done
done
