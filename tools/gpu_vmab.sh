#!/bin/bash
# view-mix backward variants: parity (test_gpu_viewmix -k view_mix) and stage times per build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in vmbase vmgw2 vmgg1 vmboth vmbase; do
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$v.so timeout -k 10 120 python -m pytest tests/test_gpu_viewmix.py -q -k view_mix -p no:cacheprovider 2>&1 | tail -1 | sed "s/^/$v /" | tee -a gpurun_out/vmab.txt || exit 1
  ANERF_LIB_PATH=$PWD/tools/ab/lib_$v.so timeout -k 10 120 python tools/viewfactor_bench.py 2>/dev/null | tail -1 | sed "s/^/$v /" | tee -a gpurun_out/vmab.txt || exit 1
done
