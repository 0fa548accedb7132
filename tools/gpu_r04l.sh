#!/bin/bash
# round 4: where the waves' cycles go (SQ counters: parked at s_waitcnt / barrier, issue-stalled,
# issuing; MFMA-busy cycles) for the training GEMMs and for render_kernel in fp16x4
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcw_gemm3 -o run --output-format csv -- python3 tools/gemm_bench.py --prec 3 --reps 5 --cases forward,input_grad,weight_grad > gpurun_out/pmcw_gemm3.log 2>&1 || { tail -20 gpurun_out/pmcw_gemm3.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcw_gemm6 -o run --output-format csv -- python3 tools/gemm_bench.py --prec 6 --reps 5 --cases forward > gpurun_out/pmcw_gemm6.log 2>&1 || { tail -20 gpurun_out/pmcw_gemm6.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcw_render -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" > gpurun_out/pmcw_render.log 2>&1 || { tail -20 gpurun_out/pmcw_render.log; exit 1; }
python tools/pmc_waves.py gpurun_out/pmcw_gemm3 gpurun_out/pmcw_gemm6 gpurun_out/pmcw_render | tee gpurun_out/r04l_pmc_waves.txt
for p in fp16x4 bf16x6; do
  PREC=$p bash tools/gpu_pmc.sh > /dev/null || exit 1
  python tools/pmc_summary.py gpurun_out gpurun_out/r04l_pmc_$p.json r04l $p > /dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r04l_pmc_$p.json')); print('$p', d['unit'], d['render_kernel_hbm_bytes_per_launch'], d['effective_clock_GHz'], d['kernel_ns'])"
done
