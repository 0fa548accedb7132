#!/bin/bash
# round 6: persistent hidden-layer forward: micro timings, in-step kernel stats, A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python tools/gemm_bench.py --prec 6 --cases forward_256,forward_persistent,copy >> $O/micro.txt 2>> $O/micro.err || exit 1
  timeout -k 10 120 python tools/gemm_bench.py --prec 3 --cases forward_256,forward_persistent >> $O/micro.txt 2>> $O/micro.err || exit 1
done
cat $O/micro.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/train_bench.py --steps 12 --warmup 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
for m in on off on off on off; do
  f=""; [ $m = off ] && f="--no-forward-persistent"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'])" | tee -a $O/ab.txt
done
