#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
ANERF_LIB_PATH=$PWD/tools/ab/lib_gpre.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread -k "(c2_ or c3_ or c4_ or t2000 or mx1 or su1 or s1_ or full_frame or config5 or near_empty) and not density and not bf16x3" > gpurun_out/ab_gpre_pytest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/ab_gpre_pytest.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
LIBS="wf gpre" PREC=bf16x6 bash tools/gpu_ab3.sh && LIBS="wf gpre" PREC=fp16x3 bash tools/gpu_ab3.sh
