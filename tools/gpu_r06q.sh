#!/bin/bash
# round 6: training step kernel stats + trace of the current tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/train_bench.py --steps 12 --warmup 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
cp $(find $O/trace -name '*kernel_stats.csv' | head -1) $O/kernel_stats.csv
cp $(find $O/trace -name '*kernel_trace.csv' | head -1) $O/kernel_trace.csv
ls -la $O
