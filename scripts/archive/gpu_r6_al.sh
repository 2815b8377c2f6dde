#!/bin/bash
# Round 6: refresh the configs[2] PMC record (profiles/pmc_traffic.json) on
# the final tree -- one FETCH_SIZE, one WRITE_SIZE and one SQ pass of
# bench.py --steps 1 --warmup 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6al}
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample --no-host-path --no-prove --no-wide --no-configs1 --sustain-seconds 0"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAVES"; do
  i=$((i + 1))
  echo "== pmc $i: $set"
  timeout -s KILL 150 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- $B > $OUT/pmc_$i.log 2>&1 || { echo "   pmc FAILED"; tail -3 $OUT/pmc_$i.log; exit 1; }
done
echo done
