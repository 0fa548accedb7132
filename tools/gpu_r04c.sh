#!/bin/bash
# round 4: layer probe sweep (L2 footprint, wave sync), in-kernel stamps (barrier wait), then tools/gpu_r04b.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 240 tools/probe/layer_probe_x6s > gpurun_out/r04c_probe.txt 2>&1 || { cat gpurun_out/r04c_probe.txt; exit 1; }
cat gpurun_out/r04c_probe.txt
ANERF_PRECISION=bf16x6 timeout -k 10 300 python tools/stamps.py 79.6 > gpurun_out/r04c_stamps_bf16x6.txt 2>&1 || { tail gpurun_out/r04c_stamps_bf16x6.txt; exit 1; }
cat gpurun_out/r04c_stamps_bf16x6.txt
TAG=r04c bash tools/gpu_r04b.sh
