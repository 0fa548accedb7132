#!/bin/bash
# training A/B at 24 and 65 joints: persistent forward + feature gradient on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
for j in 65 24; do for i in 1 2; do for m in on off; do
  f=""; [ $m = off ] && f="--no-forward-persistent"
  timeout -k 10 200 python tools/train_bench.py --joints $j --steps 20 --warmup 3 $f > $O/t${j}_$m.json 2>> $O/err || exit 1
  python -c "import json;d=json.load(open('$O/t${j}_$m.json'));print('$j $m',d['value'],d['ms_per_step'])" | tee -a $O/ab.txt
done; done; done
