#!/bin/bash
# Experiment build for kernel A/B runs (never used by tests, bench or the driver): only the config-3
# shape (W 256, multires 7) of the render / density kernels, extra -D flags from the command line.
#   bash tools/build_ab.sh NAME [-DFLAG ...]   ->  tools/ab/lib_NAME.so   (run with ANERF_LIB_PATH=...)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/ab
NAME=$1; shift
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-result"
[ -f tools/ab/gemm.o ] && [ tools/ab/gemm.o -nt a-nerf_amd/csrc/anerf_gemm.hip ] || /opt/rocm/bin/hipcc $F -c -o tools/ab/gemm.o a-nerf_amd/csrc/anerf_gemm.hip
/opt/rocm/bin/hipcc $F -DANERF_AB_FAST "$@" -c -o tools/ab/render_$NAME.o a-nerf_amd/csrc/anerf_render.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/lib_$NAME.so tools/ab/render_$NAME.o tools/ab/gemm.o
rm -f tools/ab/render_$NAME.o
