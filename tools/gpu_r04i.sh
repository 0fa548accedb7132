#!/bin/bash
# round 4: GPU tests of the product build (now with fp16x4), the fp16x4 A/B (tools/gpu_r04h.sh), its
# oracle parity on bench.py's 20 k-ray sample next to bf16x6's, then the GEMM staging-interleave A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/r04i_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/r04i_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
bash tools/gpu_r04h.sh || exit 1
for p in fp16x4 bf16x6; do
  timeout -k 10 400 python bench.py --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision $p \
      > gpurun_out/r04i_parity_$p.json 2> gpurun_out/r04i_parity_$p.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04i_parity_$p.json')); print('$p', d['value'], json.dumps(d.get('parity')))"
done
echo "== GEMM interleave: correctness (test_gpu_mlp with lib_gil1), then A/B"
ANERF_LIB_PATH=$PWD/tools/ab/lib_gil1.so timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "gemm or nerf_forward" 2>&1 | tail -3
LIBS="il0 il1" bash tools/gpu_gemm_libs.sh 2>&1 | grep -E "==|forward|input_grad" | python -c "
import sys,json
cur=None
for l in sys.stdin:
    if l.startswith('=='): cur=l.strip(); continue
    d=json.loads(l); print(cur, d['case'], d['us'], d['TFLOPs_ref'])"
exit $rc
