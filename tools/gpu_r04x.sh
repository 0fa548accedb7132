#!/bin/bash
# round 4 end: GPU tests, smoke, default bench, launcher at one rank, rocprofv3 kernel stats, density
# throughput per precision, training-step kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r04x
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['precision'], d['roofline']['frac'], d['roofline']['frac_executed'], {k: v['rays_per_s_kernel'] for k, v in (d['other_precisions'] or {}).items()}, d['training']['value'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_launch1.json 2> gpurun_out/${TAG}_launch.err || { tail -20 gpurun_out/${TAG}_launch.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
for p in fp32 bf16x6 fp16x4 fp16x3; do
  timeout -k 10 300 python tools/density_bench.py 255 $p > gpurun_out/${TAG}_density_$p.json 2>/dev/null || exit 1
  cat gpurun_out/${TAG}_density_$p.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_${TAG} -o run --output-format csv -- python3 tools/train_bench.py --steps 5 --warmup 1 > gpurun_out/${TAG}_prof_train.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/${TAG}_prof_train.log; exit 1; }
exit $rc
