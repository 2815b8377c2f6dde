#!/bin/bash
# L1/L2 request counters of the encode (one rocprofv3 --pmc pass per set).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcl2}
mkdir -p $OUT
i=0
for set in "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCP_TCC_WRITE_REQ_sum TCC_REQ_sum"; do
  i=$((i+1))
  echo "== pmc pass $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample > $OUT/pmc_$i.log 2>&1 || { echo "   FAILED"; tail -n 5 $OUT/pmc_$i.log; exit 1; }
done
echo done
