#!/bin/bash
# round 6: wave states and LDS bank conflicts of the fused hidden-layer backward (SQ counters, separate passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
C2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for n in base p4; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_g$n.so timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmcd_$n -o run --output-format csv -- python3 tools/dgw_bench.py --reps 5 --cases fused > gpurun_out/pmcd_$n.log 2>&1 || { tail -20 gpurun_out/pmcd_$n.log; exit 1; }
  ANERF_LIB_PATH=$PWD/tools/ab/lib_g$n.so timeout -s KILL 120 rocprofv3 --pmc $C2 --kernel-trace -d gpurun_out/pmcd2_$n -o run --output-format csv -- python3 tools/dgw_bench.py --reps 5 --cases fused > gpurun_out/pmcd2_$n.log 2>&1 || { tail -20 gpurun_out/pmcd2_$n.log; exit 1; }
done
python tools/pmc_waves.py gpurun_out/pmcd_base gpurun_out/pmcd_p4 | tee gpurun_out/r06e_pmc_waves.txt
