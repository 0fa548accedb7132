#!/bin/bash
# round 5: staged-encoder render throughput next to the fused kernel; the default bench of the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r05t
timeout -k 10 300 python tools/staged_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_staged_bench.txt || exit 1
timeout -k 10 500 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['traffic_source'], {k: v['rays_per_s_kernel'] for k, v in (d['other_precisions'] or {}).items()}, d['training']['value'] if d.get('training') else None)"
