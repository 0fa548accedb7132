#!/bin/bash
# view-window stage kernels across experiment builds (tools/viewfactor_bench.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in vfbase vfb64 vfb256 vfbase; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$v.so timeout -k 10 120 python tools/viewfactor_bench.py 2>/dev/null | tail -1 | sed "s/^/$v /" | tee -a gpurun_out/vfab.txt || exit 1
done
