#!/bin/bash
# Round-3 session e (product build): the default bench line, its rocprofv3 --kernel-trace --stats
# profile, and the HBM / SQ PMC passes (separate runs) for the headline bf16x6 and for fp16x3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03e}
timeout -k 10 420 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']); print(d.get('parity'))" gpurun_out/${TAG}_bench.json
TAG=$TAG PREC=bf16x6 bash tools/gpu_prof.sh || exit 1
mkdir -p gpurun_out/bf16x6 && mv gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq gpurun_out/bf16x6/
PREC=fp16x3 bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out gpurun_out/${TAG}_pmc_fp16x3.json "${TAG}" fp16x3
exit 0
