#!/bin/bash
# Experiment build of the training GEMMs (never used by tests, bench or the driver): the in-tree render
# kernels' fast A/B subset plus anerf_gemm.hip with extra -D flags.
#   bash tools/build_gemm_ab.sh NAME [-DFLAG ...]   ->  tools/ab/lib_gNAME.so   (run with ANERF_LIB_PATH=...)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/ab
NAME=$1; shift
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-result"
[ -f tools/ab/render_fast.o ] && [ tools/ab/render_fast.o -nt a-nerf_amd/csrc/anerf_render.hip ] || /opt/rocm/bin/hipcc $F -DANERF_AB_FAST -c -o tools/ab/render_fast.o a-nerf_amd/csrc/anerf_render.hip
/opt/rocm/bin/hipcc $F "$@" -c -o tools/ab/gemm_$NAME.o a-nerf_amd/csrc/anerf_gemm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/lib_g$NAME.so tools/ab/render_fast.o tools/ab/gemm_$NAME.o
rm -f tools/ab/gemm_$NAME.o
