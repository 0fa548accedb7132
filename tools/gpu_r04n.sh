#!/bin/bash
# round 4: the fp16 hidden layer alone (NP = 3, 4 products) next to the bf16x6 one, and the fp16x4
# stamps of the product schedule (persistent queues)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in h4_probe_3 h4_probe_4 power_probe_0; do timeout -k 10 120 tools/probe/$b || exit 1; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04n_layer_probe.txt
ANERF_LIB_PATH=$PWD/tools/ab/libanerf_hip_stamps.so ANERF_PRECISION=fp16x4 timeout -k 10 300 python tools/stamps.py \
    > gpurun_out/r04n_stamps_fp16x4.txt 2>&1 || { tail gpurun_out/r04n_stamps_fp16x4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r04n_stamps_fp16x4.txt
