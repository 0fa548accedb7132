#!/bin/bash
# Experiment build of the training GEMMs against the in-tree render object (a-nerf_amd/.objs, from build.py):
#   bash tools/build_dgw_ab.sh NAME [-DFLAG ...]  ->  tools/ab/lib_gNAME.so   (run with ANERF_LIB_PATH=...)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/ab
NAME=$1; shift
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-result"
R=$(ls a-nerf_amd/.objs/anerf_render.*.o | head -1)
/opt/rocm/bin/hipcc $F "$@" -c -o tools/ab/gemm_$NAME.o a-nerf_amd/csrc/anerf_gemm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/lib_g$NAME.so $R tools/ab/gemm_$NAME.o
rm -f tools/ab/gemm_$NAME.o
