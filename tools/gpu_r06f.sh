#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "backward_hidden" > gpurun_out/r06f_pytest_dgw.log 2>&1; rc=$?
tail -3 gpurun_out/r06f_pytest_dgw.log
[ $rc -eq 0 ] || exit $rc
LIBS="base bd3 bd4 p4 p1" TAG=r06f bash tools/gpu_r06c.sh
