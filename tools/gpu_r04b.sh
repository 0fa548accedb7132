#!/bin/bash
# round 4: GPU tests, the default bench (new legs: other configs, shard balance projection), and the
# launcher path at one rank (config 5, tiled pixel split + RCCL all-gather)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r04b}
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|H12" gpurun_out/${TAG}_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== bench default"
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
echo "== launcher, 1 rank"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_launch1.json 2> gpurun_out/${TAG}_launch.err || { tail -20 gpurun_out/${TAG}_launch.err; exit 1; }
cat gpurun_out/${TAG}_bench_launch1.json
exit $rc
