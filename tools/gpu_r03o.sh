#!/bin/bash
# in-kernel stamps (tools/build_stamps.sh build) for bf16x6 and fp16x3 at config 3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r03o}
for p in bf16x6 fp16x3; do
  echo "== stamps $p"
  ANERF_PRECISION=$p timeout -k 10 300 python tools/stamps.py 79.6 > gpurun_out/${TAG}_stamps_$p.txt 2>&1 || { tail gpurun_out/${TAG}_stamps_$p.txt; exit 1; }
  cat gpurun_out/${TAG}_stamps_$p.txt
done
