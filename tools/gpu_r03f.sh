#!/bin/bash
# Round-3 session f: the MLP GEMM tests at the larger shapes, and the launcher path at one rank with
# its stdout checked to be the one result line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03f}
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/${TAG}_mlp.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_mlp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 1 --steps 3 --warmup 1 --no-train > gpurun_out/${TAG}_launcher1.json 2> gpurun_out/${TAG}_launcher1.err || { tail -20 gpurun_out/${TAG}_launcher1.err; exit 1; }
echo "stdout lines: $(grep -c '' gpurun_out/${TAG}_launcher1.json)"
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['config']['workload'], d['per_rank'], d['parity']['max_abs_err'], d['parity']['ok'])" gpurun_out/${TAG}_launcher1.json
