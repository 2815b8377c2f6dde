#!/bin/bash
# Instruction-fetch counters of the encode (one rocprofv3 --pmc pass per set):
# does the first-pass kernel's code (~120 KiB) miss the instruction cache?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcic}
mkdir -p $OUT
i=0
for set in ${SETS:-"SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE"}; do
  i=$((i+1))
  echo "== pmc pass $i: $set"
  timeout -s KILL 60 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample > $OUT/pmc_$i.log 2>&1 || { echo "   FAILED"; tail -n 5 $OUT/pmc_$i.log; exit 1; }
done
echo done
