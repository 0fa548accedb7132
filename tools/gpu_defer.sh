#!/bin/bash
# deferred side-stream sync: parity (training + MLP tests) and training A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py tests/test_kinematics.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do for m in on off; do
  f=""; [ $m = off ] && f="--no-defer-sync"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'])" | tee -a $O/ab.txt
done; done
