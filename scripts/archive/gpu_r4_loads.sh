#!/bin/bash
# Round 4: request shape of the MAC's sector loads.  The load microbench
# (scripts/ubench_loads.hip) and the encode, each under the same L1/L2 request
# counters (one rocprofv3 --pmc pass per set, each under its own kill timeout).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4loads}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
echo "== ubench timing"
timeout -k 10 120 ./scripts/ubench_loads 8 5 > $OUT/ubench.log 2>&1 || { echo FAILED; cat $OUT/ubench.log; exit 1; }
cat $OUT/ubench.log
echo "== ubench stats"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/ub_stats -o run --output-format csv -- ./scripts/ubench_loads 8 2 > $OUT/ub_stats.log 2>&1 || { echo FAILED; tail -5 $OUT/ub_stats.log; exit 1; }
i=0
IFS=';' read -ra SETS <<< "${COUNTERS:-TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_FLAT_READ_WAVEFRONTS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_REQ_sum GRBM_GUI_ACTIVE}"
for set in "${SETS[@]}"; do
  i=$((i+1))
  echo "== pmc $i ubench: $set"
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/ub_pmc_$i -o run --output-format csv -- ./scripts/ubench_loads 8 1 > $OUT/ub_pmc_$i.log 2>&1 || { echo "   FAILED"; tail -5 $OUT/ub_pmc_$i.log; exit 1; }
  echo "== pmc $i encode: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/enc_pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --gib 8 --no-cpu-baseline --no-parity-sample > $OUT/enc_pmc_$i.log 2>&1 || { echo "   FAILED"; tail -5 $OUT/enc_pmc_$i.log; exit 1; }
done
echo done
