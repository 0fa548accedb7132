#!/bin/bash
# List the PMC counters rocprofv3 offers on this GPU (TCC / EA / DRAM ones shown).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1 || true
grep -o -E "(TCC|TCA|EA|MALL|DRAM|HBM)[A-Za-z0-9_]*" gpurun_out/avail.txt | sort -u | tr '\n' ' '
exit 0
