#!/bin/bash
# bf16x6 iteration: layer probes (new vs previous commit's layer), bf16x6 parity tests, bf16x6 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in ${PROBES:-layer_probe_x6_old layer_probe_x6}; do
  echo "== $b"; timeout -k 10 60 tools/probe/$b || exit 1
done
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu -k "${TESTK:-bf16x6}" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x6.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_x6.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --precision ${PREC:-bf16x6} || exit 1
exit $rc
