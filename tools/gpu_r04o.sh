#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for b in h4_probe_4 h4_probe_4ns h4_probe_4nsplit h4_probe_4nl; do echo "== $b"; timeout -k 10 120 tools/probe/$b || exit 1; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r04o_layer_probe_parts.txt
