#!/bin/bash
# fp16x3 bring-up: its parity tests, then the bench in fp16x3 (and the other modes beside it).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-h3}
timeout -k 10 600 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    -k "${K:-fp16x3 or split}" > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 400 python bench.py --precision ${PREC:-fp16x3} --no-cpu --no-tau20 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
exit $rc
