#!/bin/bash
# Round-3 session b: the H12 reference fixture on the GPU (printed per precision), the GPU test suite,
# and the launcher (pixel-shard, ray-balanced) bench path at one rank.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -q -s -m gpu -k "near_empty" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_h12.log 2>&1; rc=$?
grep -E "H12|passed|failed|Error|assert" gpurun_out/${TAG}_h12.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== launcher, 1 rank (pixel shard, ray-balanced)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 1 --steps 3 --warmup 1 --no-train > gpurun_out/${TAG}_launcher1.json 2> gpurun_out/${TAG}_launcher1.err || { tail -20 gpurun_out/${TAG}_launcher1.err; exit 1; }
cat gpurun_out/${TAG}_launcher1.json
exit $rc
