#!/bin/bash
# staged-encoder eval renders with the persistent forward on / off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python tools/staged_bench.py > $O/staged_on.txt 2>> $O/err || exit 1
cat $O/staged_on.txt
timeout -k 10 300 python -c "
import importlib, runpy, sys
importlib.import_module('a-nerf_amd.mlp').FORWARD_PERSISTENT = False
sys.argv = ['tools/staged_bench.py']
runpy.run_path('tools/staged_bench.py', run_name='__main__')
" > $O/staged_off.txt 2>> $O/err || exit 1
sed 's/^/off /' $O/staged_off.txt
for i in 1 2 3; do for m in on off; do
  f=""; [ $m = off ] && f="--no-fine-stream"
  timeout -k 10 200 python tools/train_bench.py --steps 30 --warmup 3 $f > $O/fs_$m.json 2>> $O/err || exit 1
  python -c "import json;d=json.load(open('$O/fs_$m.json'));print('fine-stream $m',d['value'],d['ms_per_step'],d['host_issue_ms_per_step'])" | tee -a $O/ab.txt
done; done
