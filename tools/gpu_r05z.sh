#!/bin/bash
# round 5: kernel stats of the training step in the view-window layout and with the full view columns
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05z
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_w -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 \
    > gpurun_out/${TAG}_w.log 2>&1 || { tail -20 gpurun_out/${TAG}_w.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_f -o run --output-format csv -- python3 tools/train_bench.py --steps 6 --warmup 2 --full-view \
    > gpurun_out/${TAG}_f.log 2>&1 || { tail -20 gpurun_out/${TAG}_f.log; exit 1; }
ls gpurun_out/${TAG}_w gpurun_out/${TAG}_f
