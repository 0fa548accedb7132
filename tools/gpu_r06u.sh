#!/bin/bash
# round 6: persistent hidden-layer forward (ABI 19): parity + training A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q -m gpu --timeout 120 --timeout-method thread -k "forward_hidden or persistent" > $O/pytest_fwd.log 2>&1 || { tail -40 $O/pytest_fwd.log; exit 1; }
tail -2 $O/pytest_fwd.log
for m in on off on off; do
  f=""; [ $m = off ] && f="--no-forward-persistent"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python tools/train_bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1 || exit 1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
