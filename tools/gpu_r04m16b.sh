#!/bin/bash
# fp16x4 forward GEMM micro-timings, the mlp/train GPU tests, then the training step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/gemm_f16_bench.py > gpurun_out/r04m16b_gemm.txt 2>&1 || { tail -20 gpurun_out/r04m16b_gemm.txt; exit 1; }
cat gpurun_out/r04m16b_gemm.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py -q -m gpu -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/r04m16b_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04m16b_pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for m in mixed mixed16; do
    timeout -k 10 200 python tools/train_bench.py --mlp $m >> gpurun_out/r04m16b_train_ab.txt 2>> gpurun_out/r04m16b_train_ab.err \
      || { tail -20 gpurun_out/r04m16b_train_ab.err; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r04m16b_train_ab.txt"):
    if l.startswith("{"):
        d = json.loads(l); print(d.get("mlp"), d.get("value"), d.get("ms_per_step"))
PY
