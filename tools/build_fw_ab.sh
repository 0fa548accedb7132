#!/bin/bash
# experiment builds of the persistent forward: bash tools/build_fw_ab.sh NAME -DFLAG... -> tools/ab/lib_gNAME.so
set -e
cd "$(dirname "$0")/.."
R=$(ls -t a-nerf_amd/.objs/anerf_render.*.o | head -1)
NAME=$1; shift
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-result"
mkdir -p tools/ab
/opt/rocm/bin/hipcc $F "$@" -c -o tools/ab/gemm_$NAME.o a-nerf_amd/csrc/anerf_gemm.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/lib_g$NAME.so $R tools/ab/gemm_$NAME.o
rm -f tools/ab/gemm_$NAME.o
