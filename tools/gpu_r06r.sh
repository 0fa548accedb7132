#!/bin/bash
# round 6: forward GEMM micro-timings (bf16x6 / bf16x3 / fp16x4) + copy floor, and mixed vs mixed16 in the step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06r
mkdir -p $O
timeout -k 10 120 python tools/gemm_f16_bench.py > $O/f16.txt 2>&1 || { tail $O/f16.txt; exit 1; }
cat $O/f16.txt
timeout -k 10 120 python tools/gemm_bench.py --prec 6 --cases forward,input_grad,copy > $O/g6.txt 2>&1 || { tail $O/g6.txt; exit 1; }
cat $O/g6.txt
for m in mixed mixed16 mixed mixed16; do
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 --mlp $m > $O/train_$m.json 2>> $O/train.err || exit 1
  python -c "import json;d=json.load(open('$O/train_$m.json'));print('$m',d['value'],d['ms_per_step'])"
done
