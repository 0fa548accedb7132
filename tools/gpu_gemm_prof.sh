#!/bin/bash
# GEMM microbenchmark + PMC counters of the training MLP kernels (separate passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-gemm}
timeout -k 10 120 python tools/gemm_bench.py --prec ${PREC:-6} | tee gpurun_out/${TAG}_bench.jsonl || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d gpurun_out/pmc_${TAG}_a -o run --output-format csv -- python3 tools/gemm_bench.py --reps 2 > gpurun_out/pmc_${TAG}_a.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_a.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_${TAG}_b -o run --output-format csv -- python3 tools/gemm_bench.py --reps 2 > gpurun_out/pmc_${TAG}_b.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_b.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_${TAG}_f -o run --output-format csv -- python3 tools/gemm_bench.py --reps 2 > gpurun_out/pmc_${TAG}_f.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_f.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_${TAG}_w -o run --output-format csv -- python3 tools/gemm_bench.py --reps 2 > gpurun_out/pmc_${TAG}_w.log 2>&1 || { tail -5 gpurun_out/pmc_${TAG}_w.log; exit 1; }
echo done
