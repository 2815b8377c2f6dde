#!/bin/bash
# Round 4, second call: L1/TA request counters of the first pass with whole-line
# vs sector-shaped MAC loads, the cold-call phase trace at configs[3], rocprof
# stats, and the full default bench lines (c3 with CPU rows, c5 with the native
# prove row).  Every step under its own limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4b}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample --gib 16"
i=0
IFS=';' read -ra SETS <<< "${COUNTERS:-TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD;FETCH_SIZE GRBM_GUI_ACTIVE}"
for set in "${SETS[@]}"; do
  i=$((i+1))
  for v in line sector; do
    if [ $v = sector ]; then export HB_MFMA_SECTOR_LOADS=1; else unset HB_MFMA_SECTOR_LOADS; fi
    echo "== pmc $v $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_${v}_$i -o run --output-format csv -- $B > $OUT/pmc_${v}_$i.log 2>&1 || { echo "   pmc FAILED"; tail -3 $OUT/pmc_${v}_$i.log; exit 1; }
  done
done
unset HB_MFMA_SECTOR_LOADS
HB_TRACE_PHASES=1 step c4_cold_trace 300 python3 -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample || exit 1
step stats_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/stats_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
step bench_c5 300 python3 -u bench.py --config c5 || exit 1
step bench_c3 600 python3 -u bench.py || exit 1
echo done
