set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo | grep -m1 -i "gfx950" > gpurun_out/rocminfo.txt || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -p no:cacheprovider > gpurun_out/t1.log 2>&1
echo "pytest rc=$?"
tail -30 gpurun_out/t1.log
