#!/bin/bash
# GEMM numerics tests, then the microbenchmark.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-gq}
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/gemm_bench.py --prec 6 | tee gpurun_out/${TAG}_bench.jsonl || exit 1
timeout -k 10 120 python tools/gemm_bench.py --prec 3 | tee -a gpurun_out/${TAG}_bench.jsonl || exit 1
