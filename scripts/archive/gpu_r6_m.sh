#!/bin/bash
# Round 6: PMC of hb_wmac_kernel (cxx 1024-bit encode: the MAC dominates), one
# counter set per pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6m}
mkdir -p $OUT
i=0
for set in "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:2:cxx > $OUT/pmc_$i.log 2>&1 || { echo "   pmc FAILED"; tail -5 $OUT/pmc_$i.log; exit 1; }
done
echo done
