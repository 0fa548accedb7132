#!/bin/bash
# round 5: the view-window training layout (anerf.h ANERF_ENC_VIEW_WINDOWS): training parity in both layouts, the
# training-step A/B (interleaved) and the kernel stats of the new default
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05x
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_mlp.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
for i in 1 2; do
  for v in "" "--full-view"; do
    timeout -k 10 200 python tools/train_bench.py --steps 20 $v 2>/dev/null | tail -1 | sed "s/^/[${v:-windows}] /" | tee -a gpurun_out/${TAG}_train_ab.txt || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 \
    > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/${TAG}_train_kernel_stats.csv
head -12 gpurun_out/${TAG}_train_kernel_stats.csv | cut -c1-160
