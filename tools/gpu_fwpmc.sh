#!/bin/bash
# PMC passes over the persistent forward micro (forward_persistent, M = 163,840, bf16x6), one counter set a pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
B="tools/gemm_bench.py --prec 6 --cases forward_persistent --reps 10"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace -d $O/pa -o run --output-format csv -- python3 $B > $O/pa.log 2>&1 || { tail -5 $O/pa.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d $O/pb -o run --output-format csv -- python3 $B > $O/pb.log 2>&1 || { tail -5 $O/pb.log; exit 1; }
find $O -name "*counter_collection.csv" | head
