#!/bin/bash
# round 6: CPU-side profile of the training step (cProfile over tools/train_bench.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m cProfile -o gpurun_out/r06j_train.prof tools/train_bench.py --steps 30 --warmup 3 > gpurun_out/r06j_train.json 2> gpurun_out/r06j_train.err || { tail -5 gpurun_out/r06j_train.err; exit 1; }
python - <<'PY' > gpurun_out/r06j_cprofile.txt
import pstats
p = pstats.Stats("gpurun_out/r06j_train.prof")
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(60)
PY
head -80 gpurun_out/r06j_cprofile.txt | tail -60
