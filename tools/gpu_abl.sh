#!/bin/bash
# Ablations of the training GEMM (ANERF_GEMM_DBG bits, see anerf_gemm.hip NTArgs::dbg).
cd "$GRAFT_REPO_ROOT"
for d in 0 1 2 4 6 7; do echo "dbg=$d"; ANERF_GEMM_DBG=$d timeout -k 10 60 python tools/gemm_bench.py --prec 6 | grep forward || exit 1; done
