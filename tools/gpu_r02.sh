#!/bin/bash
# Round-2 GPU session: the whole -m gpu suite, then the default bench (with CPU baseline + parity leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
[ -n "$NOBENCH" ] && exit $rc
echo "== bench"
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
exit $rc
