#!/bin/bash
# HBM traffic of render_kernel: FETCH_SIZE and WRITE_SIZE in separate --pmc passes (TCC slots).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision ${PREC:-fp16x3} > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision ${PREC:-fp16x3} > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" --precision ${PREC:-fp16x3} > gpurun_out/pmc_sq.log 2>&1 || { tail -20 gpurun_out/pmc_sq.log; exit 1; }
find gpurun_out/pmc_* -name "*.csv" | head -20
