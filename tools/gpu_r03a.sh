#!/bin/bash
# Round-3 first box session: quick per-precision bench lines, the GPU test suite, in-kernel stamps
# for bf16x6 and fp16x3 (tools/ab/libanerf_hip_stamps.so from tools/build_stamps.sh).  Each GPU step
# has its own limit; a crash or timeout ends the session.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r03a}
for p in ${PRECS:-bf16x6 fp16x3}; do
  echo "== bench $p"
  timeout -k 10 300 python bench.py --no-cpu --no-train --no-tau20 --also "" --precision $p > gpurun_out/${TAG}_bench_$p.json 2> gpurun_out/${TAG}_bench_$p.err || { tail -20 gpurun_out/${TAG}_bench_$p.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac_executed'])" gpurun_out/${TAG}_bench_$p.json
done
if [ -z "$NO_TESTS" ]; then
  echo "== pytest"
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?
  grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | tail -25
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for p in ${STAMP_PRECS:-bf16x6}; do
  echo "== stamps $p"
  ANERF_PRECISION=$p timeout -k 10 300 python tools/stamps.py 79.6 > gpurun_out/${TAG}_stamps_$p.txt 2>&1 || { tail gpurun_out/${TAG}_stamps_$p.txt; exit 1; }
  cat gpurun_out/${TAG}_stamps_$p.txt
done
for p in ${PMC_PRECS:-bf16x6}; do
  echo "== pmc $p"
  i=0
  for set in "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU" \
             "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace -d gpurun_out/${TAG}_pmc_${p}_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-train --no-tau20 --also "" --precision $p > gpurun_out/${TAG}_pmc_${p}_$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc_${p}_$i.log; exit 1; }
  done
  T=$(python -c "print({'fp32': 0, 'bf16x3': 1, 'bf16x6': 2, 'fp16x3': 3}['$p'])")
  for f in gpurun_out/${TAG}_pmc_${p}_*/run_counter_collection.csv; do grep "render_kernel<256, 7, $T>" "$f" | awk -F'","' '{print $16, $17}' | sort | awk '{a[$1]+=$2} END {for (k in a) printf "%s %.6g\n", k, a[k]}'; done
done
exit ${rc:-0}
