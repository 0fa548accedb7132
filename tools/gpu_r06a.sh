#!/bin/bash
# round 6 first run: GPU suite, smoke, default bench, rocprofv3 kernel stats of the shipped build, PMC passes of the
# timed call (bench --no-tally), training bench with the PoseOptLayer step vs the delta leaf
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r06a
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['roofline']['frac'], d['training']['value'] if d.get('training') else None)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-tau20 --no-train --no-balance --no-tally --other-configs= --also= > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
PREC=fp16x4 timeout -k 10 900 bash tools/gpu_pmc.sh || exit 1
for p in kinematic delta kinematic delta; do
  timeout -k 10 200 python tools/train_bench.py --steps 20 --pose $p 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$p', d['value'], d['ms_per_step'])" | tee -a gpurun_out/${TAG}_train_pose_ab.txt || exit 1
done
