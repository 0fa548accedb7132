#!/bin/bash
# MFMA-busy and clock of the persistent forward micro per build (PMC).  usage: bash tools/gpu_fwpmc2.sh <tag> <libs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
for v in base "$@"; do
  L=""; [ $v != base ] && L=tools/ab/lib_g$v.so
  ANERF_LIB_PATH=$L timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA --kernel-trace -d $O/$v -o run --output-format csv -- python3 tools/gemm_bench.py --prec 6 --cases forward_persistent --reps 10 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  python3 - $O/$v/run_counter_collection.csv $v <<'PY'
import csv, sys, collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(list); dur=[]
for r in rows:
    if 'mlp_fwd' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
        dur.append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
a={k:sum(v)/len(v) for k,v in agg.items()}
us=sorted(dur)[len(dur)//2]
cyc=a['GRBM_GUI_ACTIVE']/8
print(sys.argv[2], 'us', round(us,1), 'GHz', round(cyc/us/1e3,3), 'mfma_busy', round(a['SQ_VALU_MFMA_BUSY_CYCLES']/1024/cyc,3))
PY
done
