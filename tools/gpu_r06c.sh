#!/bin/bash
# round 6: fused hidden-layer backward A/B microbenchmarks (ring depth, probes) vs the two GEMMs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 1 2; do
  for n in ${LIBS:-base bd3 p1 p2 p4}; do
    echo -n "$n " | tee -a gpurun_out/${TAG:-r06c}_dgw_ab.txt
    ANERF_LIB_PATH=$PWD/tools/ab/lib_g$n.so timeout -k 10 120 python tools/dgw_bench.py --cases fused$([ $n = base ] && echo ",two_seq,two_streams") | tee -a gpurun_out/${TAG:-r06c}_dgw_ab.txt || exit 1
  done
done
