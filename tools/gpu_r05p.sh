#!/bin/bash
# round 5: the product build with the composite's scalar wave index: GPU tests, the fp16x4 PMC passes
# (HBM traffic per call), the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05p
timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -15
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
PREC=fp16x4 bash tools/gpu_pmc.sh > /dev/null || exit 1
python tools/pmc_summary.py gpurun_out gpurun_out/${TAG}_pmc_fp16x4.json "$TAG" fp16x4 > /dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/${TAG}_pmc_fp16x4.json')); print('fp16x4', d['render_kernel_hbm_bytes_per_launch'], d['FETCH_SIZE_KB_per_launch'], d['WRITE_SIZE_KB_per_launch'], d['effective_clock_GHz'], d['kernel_ns'])"
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['traffic_source'], {k: v['rays_per_s_kernel'] for k, v in (d['other_precisions'] or {}).items()}, d['training']['value'] if d.get('training') else None)"
