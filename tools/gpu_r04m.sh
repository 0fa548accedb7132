#!/bin/bash
# round 4: training NT GEMM with the B-fragment ring 4 deep (prefetch 3 k16-steps ahead) vs 2 deep:
# correctness, GEMM microbench A/B, training-step A/B, SQ wave states of the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/r04m_gemm_bd.txt
echo "== bd4 correctness" | tee $O
ANERF_LIB_PATH=$PWD/tools/ab/lib_gbd4.so timeout -k 10 300 python -m pytest tests/test_gpu_mlp.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread 2>&1 | tail -2 | tee -a $O
LIBS="bd2 bd4" CASES=forward,input_grad bash tools/gpu_gemm_libs.sh 2>&1 | grep -v amdgpu.ids | tee -a $O || exit 1
for r in 1 2; do
  for l in bd2 bd4; do
    echo "== train $l" | tee -a $O
    ANERF_LIB_PATH=$PWD/tools/ab/lib_g$l.so timeout -k 10 300 python tools/train_bench.py --steps 10 2>/dev/null | tail -1 | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'])" | tee -a $O || exit 1
  done
done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
ANERF_LIB_PATH=$PWD/tools/ab/lib_gbd4.so timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcw_bd4 -o run --output-format csv -- python3 tools/gemm_bench.py --prec 3 --reps 5 --cases forward,input_grad,weight_grad > gpurun_out/pmcw_bd4.log 2>&1 || { tail -20 gpurun_out/pmcw_bd4.log; exit 1; }
python tools/pmc_waves.py gpurun_out/pmcw_bd4 | tee -a $O
