#!/bin/bash
# round 5 end: bench.py under the launcher at 1 rank (the driver's N > 1 command shape) on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=r05zr
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_launch1.json 2> gpurun_out/${TAG}_launch.err || { tail -20 gpurun_out/${TAG}_launch.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_launch1.json')); print(d['value'], d['n_gpus'], d['config'].get('parallelism'), d.get('scaling'))"
