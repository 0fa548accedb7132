#!/bin/bash
# round 6: training step -- host issue time and the GPU's busy union from a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 > $O/train.json 2> $O/train.err || exit 1
cat $O/train.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/train_bench.py --steps 12 --warmup 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
f=$(find $O/trace -name '*kernel_trace.csv' | head -1)
cp "$f" $O/kernel_trace.csv
python tools/busy_union.py $O/kernel_trace.csv > $O/busy.txt && cat $O/busy.txt
