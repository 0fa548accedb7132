set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in 0 1 2 3; do echo "== probe v$v"; timeout -k 10 120 ./tools/probe/layer_probe_x6_v$v || exit 1; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -q -s -m gpu -k "near_empty" -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r03c_h12.log 2>&1; rc=$?
grep -E "H12|passed|failed" gpurun_out/r03c_h12.log | tail -6
exit 0
