#!/bin/bash
# round 6: fine pass on its own stream (coarse / fine backward overlap): parity + training A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_mlp.py tests/test_kinematics.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in on off on off; do
  f=""; [ $m = off ] && f="--no-fine-stream"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'],d['host_issue_ms_per_step'])"
done
timeout -k 10 200 python tools/train_bench.py --joints 65 --steps 20 --warmup 3 > $O/train65.json 2>> $O/train.err || exit 1
python -c "import json;d=json.load(open('$O/train65.json'));print('65',d['value'],d['ms_per_step'])"
