#!/bin/bash
# round 6: persistent hidden-layer forward iteration: parity, micro timings, in-step kernel stats, A/B
# usage: bash tools/gpu_fw.sh <tag> [ab-pairs]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
N=${2:-2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp.py -x -q -m gpu --timeout 120 --timeout-method thread -k "forward_hidden or forward_layer or persistent" > $O/pytest_fwd.log 2>&1 || { tail -40 $O/pytest_fwd.log; exit 1; }
tail -1 $O/pytest_fwd.log
for r in 1 2; do
  timeout -k 10 120 python tools/gemm_bench.py --prec 6 --cases forward_256,forward_persistent >> $O/micro.txt 2>> $O/micro.err || exit 1
done
cut -c1-120 $O/micro.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/train_bench.py --steps 12 --warmup 3 > $O/trace.log 2>&1 || { tail $O/trace.log; exit 1; }
grep -h "mlp_fwd_kernel\|mlp_nt_kernel<3, 1" $O/trace/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
for i in $(seq $N); do for m in on off; do
  f=""; [ $m = off ] && f="--no-forward-persistent"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'])" | tee -a $O/ab.txt
done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py tests/test_gpu_train.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
