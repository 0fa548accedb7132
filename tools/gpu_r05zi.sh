#!/bin/bash
# view-window layout with the pre-activation accumulate: GEMM + view tests, stage times, training A/B, kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05zi}
timeout -k 10 600 python -u -m pytest tests/test_gpu_viewmix.py tests/test_gpu_mlp.py tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 120 python tools/viewfactor_bench.py 2>/dev/null | tail -1 | tee gpurun_out/${TAG}_stages.txt || exit 1
for i in 1 2; do
  for v in "" "--no-view-side"; do
    timeout -k 10 200 python tools/train_bench.py --steps 20 $v 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('${v:-windows}', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_train_ab.txt || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_w -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 \
    > gpurun_out/${TAG}_w.log 2>&1 || { tail -20 gpurun_out/${TAG}_w.log; exit 1; }
echo done
