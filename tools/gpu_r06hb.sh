#!/bin/bash
# final tree: the training step's HBM bytes (PMC FETCH_SIZE / WRITE_SIZE, separate passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06hb
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_f -o run --output-format csv -- python3 tools/train_bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_f.log 2>&1 || { tail -5 gpurun_out/${TAG}_f.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_w -o run --output-format csv -- python3 tools/train_bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_w.log 2>&1 || { tail -5 gpurun_out/${TAG}_w.log; exit 1; }
python tools/pmc_train_bytes.py gpurun_out/${TAG}_f gpurun_out/${TAG}_w > gpurun_out/${TAG}_train_hbm_bytes.json && head -4 gpurun_out/${TAG}_train_hbm_bytes.json
