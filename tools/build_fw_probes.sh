#!/bin/bash
# experiment builds of the persistent forward's timing probes (ANERF_FW_PROBE 1-4) -> tools/ab/lib_gfwp{1..4}.so
set -e
cd "$(dirname "$0")/.."
R=$(ls -t a-nerf_amd/.objs/anerf_render.*.o | head -1)
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -Wno-unused-result"
mkdir -p tools/ab
for p in 1 2 3 4; do
  /opt/rocm/bin/hipcc $F -DANERF_FW_PROBE=$p -c -o tools/ab/gemm_fwp$p.o a-nerf_amd/csrc/anerf_gemm.hip &
done
wait
for p in 1 2 3 4; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/lib_gfwp$p.so $R tools/ab/gemm_fwp$p.o
  rm -f tools/ab/gemm_fwp$p.o
done
