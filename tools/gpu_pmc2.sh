#!/bin/bash
# Extended PMC passes for render_kernel: MFMA busy / waits, instruction cache, VALU mix.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH" \
           "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/pmc2_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/pmc2_$i.log 2>&1 || { tail -20 gpurun_out/pmc2_$i.log; exit 1; }
done
for f in gpurun_out/pmc2_*/run_counter_collection.csv; do grep render_kernel "$f" | awk -F'","' '{print $16, $17}' | sort | awk '{a[$1]+=$2} END {for (k in a) printf "%s %.6g\n", k, a[k]}'; done
