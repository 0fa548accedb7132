#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r04f.sh; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r04g.sh || exit 1
exit $rc
