#!/bin/bash
# round 6: 65-joint training in the view-window layout (padded rows): view_mix + training parity, then the A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_viewmix.py tests/test_gpu_train.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in win full win full; do
  f=""; [ $m = full ] && f="--full-view"
  timeout -k 10 200 python tools/train_bench.py --joints 65 --steps 20 --warmup 3 $f > $O/train65_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train65_$m.json'));print('$m',d['value'],d['ms_per_step'],d['view_layout'])"
done
