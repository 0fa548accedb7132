#!/bin/bash
# round 6: fused backward with the side-stream slab reduce -- MLP / train / kinematics GPU tests, training A/B,
# the training step's kernel stats and HBM bytes (PMC FETCH_SIZE / WRITE_SIZE, separate passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06h
timeout -k 10 900 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py tests/test_kinematics.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.log
[ $rc -eq 0 ] || exit $rc
for v in fused two fused two; do
  f=""; [ $v = two ] && f="--no-fused-backward"
  timeout -k 10 200 python tools/train_bench.py --steps 20 $f 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_train_ab.txt || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_tprof -o run --output-format csv -- python3 tools/train_bench.py --steps 10 --warmup 2 > gpurun_out/${TAG}_tprof.log 2>&1 || { tail -5 gpurun_out/${TAG}_tprof.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_f -o run --output-format csv -- python3 tools/train_bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_f.log 2>&1 || { tail -5 gpurun_out/${TAG}_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_w -o run --output-format csv -- python3 tools/train_bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_w.log 2>&1 || { tail -5 gpurun_out/${TAG}_w.log; exit 1; }
python tools/pmc_train_bytes.py gpurun_out/${TAG}_f gpurun_out/${TAG}_w > gpurun_out/${TAG}_train_hbm_bytes.json && head -5 gpurun_out/${TAG}_train_hbm_bytes.json
