#!/bin/bash
# Diagnostics for one precision mode: in-kernel stamps (phase shares) and L2/VALU PMC passes of
# render_kernel.  Needs tools/libanerf_hip_stamps.so (tools/build_stamps.sh) built beforehand.
#   PREC=bf16x3 bash tools/gpu_diag.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
PREC=${PREC:-fp32}
export ANERF_PRECISION=$PREC
timeout -k 10 300 python tools/stamps.py 79.6 > gpurun_out/stamps_$PREC.txt 2>&1 || { tail gpurun_out/stamps_$PREC.txt; exit 1; }
cat gpurun_out/stamps_$PREC.txt
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/diag_${PREC}_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --precision $PREC > gpurun_out/diag_${PREC}_$i.log 2>&1 || { tail -20 gpurun_out/diag_${PREC}_$i.log; exit 1; }
done
for f in gpurun_out/diag_${PREC}_*/run_counter_collection.csv; do grep render_kernel "$f" | awk -F'","' '{print $16, $17}' | sort | awk '{a[$1]+=$2} END {for (k in a) printf "%s %.6g\n", k, a[k]}'; done
