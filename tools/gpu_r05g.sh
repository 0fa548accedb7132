#!/bin/bash
# round 5: render-kernel HBM writes per launch: WRITE_SIZE and the EA write requests,
# separate --pmc passes over tools/write_probe.py (3 calls with the coarse -> fine z hand-off, 3 without)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r05g
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${T}_w -o run --output-format csv -- python3 tools/write_probe.py > gpurun_out/${T}_w.log 2>&1 || { tail -20 gpurun_out/${T}_w.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --kernel-trace -d gpurun_out/${T}_ea -o run --output-format csv -- python3 tools/write_probe.py > gpurun_out/${T}_ea.log 2>&1 || { tail -20 gpurun_out/${T}_ea.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_FLAT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVES --kernel-trace -d gpurun_out/${T}_sq -o run --output-format csv -- python3 tools/write_probe.py > gpurun_out/${T}_sq.log 2>&1 || { tail -20 gpurun_out/${T}_sq.log; exit 1; }
tail -1 gpurun_out/${T}_w.log
# the fp16x4 stamps of the product schedule (diagnostic build, tools/build_stamps.sh)
ANERF_LIB_PATH=$PWD/tools/ab/libanerf_hip_stamps.so ANERF_PRECISION=fp16x4 timeout -k 10 300 python tools/stamps.py \
    > gpurun_out/${T}_stamps_fp16x4.txt 2>&1 || { tail gpurun_out/${T}_stamps_fp16x4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_stamps_fp16x4.txt | tail -30
