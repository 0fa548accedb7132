#!/bin/bash
# nan fill through LDS: the GPU tests that cover near/far and the NaN fill, training parity, the step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05zj
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train.py tests/test_gpu_boxes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for i in 1 2; do
  timeout -k 10 200 python tools/train_bench.py --steps 20 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('windows', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_train.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_w -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 \
    > gpurun_out/${TAG}_w.log 2>&1 || { tail -20 gpurun_out/${TAG}_w.log; exit 1; }
grep nan_fill gpurun_out/${TAG}_w/run_kernel_stats.csv | cut -c1-200
