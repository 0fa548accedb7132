#!/bin/bash
# HBM traffic and instruction mix of render_kernel on the timed render_rays call: FETCH_SIZE, WRITE_SIZE and the
# SQ counters in separate --pmc passes (TCC slots), each over `bench.py --no-tally` (warmup + timed step only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${PREC:-fp16x4}
B="bench.py --steps 1 --warmup 1 --no-cpu --no-tau20 --no-train --no-balance --no-tally --other-configs= --also= --precision $P"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 $B > gpurun_out/pmc_fetch.log 2>&1 || { tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python3 $B > gpurun_out/pmc_write.log 2>&1 || { tail -20 gpurun_out/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_sq -o run --output-format csv -- python3 $B > gpurun_out/pmc_sq.log 2>&1 || { tail -20 gpurun_out/pmc_sq.log; exit 1; }
find gpurun_out/pmc_* -name "*.csv" | head -20
