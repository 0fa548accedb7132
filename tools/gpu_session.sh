#!/bin/bash
# GPU-box session: bench (all precisions + the default line with the CPU baseline), parity tests,
# density bench, rocprofv3 kernel stats of the default bench, HBM PMC passes (default precision),
# training bench + its kernel stats.  Each GPU step has its own limit; a crash/timeout ends the
# session (test failures, rc 1, do not).
#   TAG=r01_v6 bash tools/gpu_session.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
for p in ${PRECS:-bf16x6 fp32 bf16x3}; do
  echo "== bench $p"
  timeout -k 10 300 python bench.py --no-cpu --also "" --precision $p > gpurun_out/${TAG}_bench_$p.json 2> gpurun_out/bench_$p.err || { tail -20 gpurun_out/bench_$p.err; exit 1; }
  cat gpurun_out/${TAG}_bench_$p.json
done
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_gpu.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
[ -n "$QUICK" ] && exit $rc
echo "== bench (default, with CPU baseline)"
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
for p in fp32 bf16x6; do
  echo "== density $p"
  timeout -k 10 300 python tools/density_bench.py 255 $p > gpurun_out/${TAG}_density_$p.json 2> gpurun_out/density.err || { tail -20 gpurun_out/density.err; exit 1; }
  cat gpurun_out/${TAG}_density_$p.json
done
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --also "" > gpurun_out/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*stats*"
echo "== pmc"
for p in ${PMC_PRECS:-bf16x6}; do
  PREC=$p bash tools/gpu_pmc.sh || exit 1
done
echo "== configs 2 and 4"
timeout -k 10 300 python bench.py --no-cpu --also "" --joints 65 > gpurun_out/${TAG}_bench_cfg4_joints65.json 2> gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu --also "" --res 256 --importance 0 > gpurun_out/${TAG}_bench_cfg2_res256.json 2> gpurun_out/cfg.err || { tail -20 gpurun_out/cfg.err; exit 1; }
cat gpurun_out/${TAG}_bench_cfg4_joints65.json gpurun_out/${TAG}_bench_cfg2_res256.json
echo "== dataset ray sampler"
timeout -k 10 200 python tools/dataset_bench.py > gpurun_out/${TAG}_dataset_bench.json 2> gpurun_out/ds.err || { tail -20 gpurun_out/ds.err; exit 1; }
cat gpurun_out/${TAG}_dataset_bench.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ds_${TAG} -o run --output-format csv -- python3 tools/dataset_bench.py > gpurun_out/prof_ds.log 2>&1 || { echo "rocprof dataset failed"; tail -20 gpurun_out/prof_ds.log; exit 1; }
echo "== train"
timeout -k 10 300 python tools/train_bench.py > gpurun_out/${TAG}_train_bench.json 2> gpurun_out/train.err || { tail -20 gpurun_out/train.err; exit 1; }
cat gpurun_out/${TAG}_train_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train_${TAG} -o run --output-format csv -- python3 tools/train_bench.py --steps 5 --warmup 1 > gpurun_out/prof_train.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/prof_train.log; exit 1; }
exit $rc
