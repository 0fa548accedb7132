#!/bin/bash
# Profiles of the default bench: rocprofv3 kernel stats, then the HBM / SQ PMC passes (separate runs,
# tools/gpu_pmc.sh) for the headline precision.  TAG names the output.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r02}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu --no-tau20 --also "" > gpurun_out/prof_${TAG}.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_${TAG}.log; exit 1; }
grep '^{' gpurun_out/prof_${TAG}.log > gpurun_out/prof_${TAG}_bench.json
find gpurun_out/prof_${TAG} -name "*stats*"
PREC=${PREC:-fp16x3} bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out gpurun_out/${TAG}_pmc_${PREC:-fp16x3}.json "${TAG}" ${PREC:-fp16x3}
