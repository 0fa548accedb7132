#!/bin/bash
# GPU-box session: parity tests, bench (both precisions), density bench, rocprofv3 kernel stats.
# Each GPU step has its own limit; the first failure ends the session.
#   TAG=r01_v6 bash tools/gpu_session.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
echo "== bench"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
for p in fp32 bf16x3; do
  echo "== bench $p"
  timeout -k 10 300 python bench.py --no-cpu --precision $p > gpurun_out/${TAG}_bench_$p.json 2> gpurun_out/bench_$p.err || { tail -20 gpurun_out/bench_$p.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$p.json
done
echo "== density"
timeout -k 10 300 python tools/density_bench.py > gpurun_out/${TAG}_density.json 2> gpurun_out/density.err || { tail -20 gpurun_out/density.err; exit 1; }
cat gpurun_out/${TAG}_density.json
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*stats*"
