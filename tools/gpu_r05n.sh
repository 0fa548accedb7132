#!/bin/bash
# round 5: PMC passes of the default bench (fp16x4, bf16x6) and the fp16x4 stamps (diagnostic build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r05n}
for p in fp16x4 bf16x6; do
  PREC=$p bash tools/gpu_pmc.sh || exit 1
  python tools/pmc_summary.py gpurun_out gpurun_out/${TAG}_pmc_$p.json "$TAG" $p > /dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${TAG}_pmc_$p.json')); print('$p', d['render_kernel_hbm_bytes_per_launch'], d['effective_clock_GHz'], d['kernel_ns'])"
done
ANERF_LIB_PATH=$PWD/tools/ab/libanerf_hip_stamps.so ANERF_PRECISION=fp16x4 timeout -k 10 300 python tools/stamps.py \
    > gpurun_out/${TAG}_stamps_fp16x4.txt 2>&1 || { tail gpurun_out/${TAG}_stamps_fp16x4.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_stamps_fp16x4.txt | tail -30
