#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|WAIT_INST|INST_LEVEL|VALU_MFMA|MFMA_BUSY|SQ_BUSY_CU|WAIT_ANY|SQ_INSTS_SALU|SQ_INSTS_LDS|SQ_INSTS_VMEM" gpurun_out/avail.txt | head -60
