#!/bin/bash
# round 5 product run: GPU tests, smoke, the default bench, the launcher at one rank, rocprofv3 kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05m}
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== smoke"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -3 gpurun_out/${TAG}_smoke.log
echo "== bench default"
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['precision'], d['roofline']['frac'], d['roofline']['frac_executed'], {k: v['rays_per_s_kernel'] for k, v in (d['other_precisions'] or {}).items()}, d['training']['value'] if d.get('training') else None, d['cpu_baseline'])"
echo "== launcher, 1 rank"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 1 --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_launch1.json 2> gpurun_out/${TAG}_launch.err || { tail -20 gpurun_out/${TAG}_launch.err; exit 1; }
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-tau20 --no-train --no-balance --other-configs "" --also "" > gpurun_out/${TAG}_prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*stats*"
exit $rc
