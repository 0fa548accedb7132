#!/bin/bash
# Diagnostic build with in-kernel s_memtime stamps (tools/stamps.py); never used by tests or bench.
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize \
    -fPIC -shared -Wno-unused-result -DANERF_STAMPS -o tools/ab/libanerf_hip_stamps.so a-nerf_amd/csrc/anerf_render.hip a-nerf_amd/csrc/anerf_gemm.hip
