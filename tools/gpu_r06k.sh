#!/bin/bash
# round 6: full GPU suite + smoke + default bench (render + 24/65-joint training legs) + pose-index A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/r06k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
for m in dev host dev host; do
  f=""; [ $m = host ] && f="--host-index"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'])"
done
