#!/bin/bash
# fp16x4 training forward ("mixed16"): GEMM / network / training-golden tests, then the training step A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04m16
true || timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py -q -m gpu -p no:cacheprovider \
    --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
rc=0
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
for r in 1 2; do
  for m in mixed mixed16; do
    timeout -k 10 200 python tools/train_bench.py --mlp $m >> gpurun_out/${TAG}_train_ab.txt 2>> gpurun_out/${TAG}_train_ab.err \
      || { tail -20 gpurun_out/${TAG}_train_ab.err; exit 1; }
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/r04m16_train_ab.txt"):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l); print(d.get("mlp"), d.get("value"), d.get("ms_per_step"))
PY
exit $rc
