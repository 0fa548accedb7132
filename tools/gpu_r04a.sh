#!/bin/bash
# round 4: H12 per-sample diagnosis against the reference's spread fixture; multi-GPU shard balance on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/diag_h12.py fp32 bf16x6 fp16x3 > gpurun_out/r04a_diag_h12.txt 2>&1 || { tail -20 gpurun_out/r04a_diag_h12.txt; exit 1; }
cat gpurun_out/r04a_diag_h12.txt
timeout -k 10 400 python -u tools/shard_balance.py --precision bf16x6 > gpurun_out/r04a_shard_balance.jsonl 2> gpurun_out/r04a_shard_balance.err || { tail -20 gpurun_out/r04a_shard_balance.err; exit 1; }
cat gpurun_out/r04a_shard_balance.jsonl
