#!/bin/bash
# GPU parity tests, then bench of each precision with the two-launch schedule (default) and the
# fused one-launch schedule (ANERF_FUSED_PASSES=1) for A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -q -x -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for p in ${PRECS:-bf16x6 fp32 bf16x3}; do
  for f in 0 1; do
    echo "== $p fused=$f"
    ANERF_FUSED_PASSES=$f timeout -k 10 300 python bench.py --no-cpu --precision $p > gpurun_out/ab_${p}_$f.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_${p}_$f.json'));print(d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])"
  done
done
exit $rc
