#!/bin/bash
# round 6: bound-based fp16 scale (ANERF_H3_BOUND) A/B on config 3, fp16x4 (experiment builds tools/build_ab.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/${TAG:-r06i}_ab.txt
for r in 1 2 3; do
  for n in ${LIBS:-h3b0 h3b1}; do
    c="--no-cpu"; [ $r = 1 ] && c=""
    timeout -k 10 300 python bench.py --lib tools/ab/lib_$n.so $c --no-tau20 --no-train --no-balance --other-configs= --also= --precision ${PREC:-fp16x4} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -5 gpurun_out/ab_$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); p=d.get('parity') or {}; print('$n', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac_executed'], p.get('max_abs_err'))" | tee -a $O
  done
done
