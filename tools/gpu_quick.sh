#!/bin/bash
# GPU tests + bench + density bench + stamps diagnostic (no rocprof)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 300 python tools/density_bench.py > gpurun_out/density.json 2> gpurun_out/density.err || { tail -20 gpurun_out/density.err; exit 1; }
cat gpurun_out/density.json
timeout -k 10 300 python tools/stamps.py 79.6 > gpurun_out/stamps.txt 2>&1 || { tail gpurun_out/stamps.txt; exit 1; }
cat gpurun_out/stamps.txt
