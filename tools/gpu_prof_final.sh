#!/bin/bash
# rocprofv3 kernel stats of the final tree: the bench's render step and training leg (no CPU / tau20 / balance / other
# configs / other precisions)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-tau20 --no-balance --no-tally --other-configs= --also= > $O/bench.json 2> $O/prof.log || { tail -20 $O/prof.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],d['training']['value'])"
