#!/bin/bash
# Round-3 phase-cost ablations of the encode (wrong-tag experiment builds, see
# hb_lane.hpp) against the in-tree build, then PMC passes over the T-table /
# bitsliced / mixed AES microbench (why the VALU engine does not add up).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3abl}
mkdir -p $OUT
TAG=${TAG:-r3abl} VARIANTS="${VARIANTS:-base nosha nomfma nold nofin}" ROUNDS=${ROUNDS:-2} \
  COUNTERS="${COUNTERS:-GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES}" \
  PMCVARIANTS="${PMCVARIANTS:-base}" bash scripts/gpu_ab.sh || exit 1
if [ -z "$NOBS" ]; then
  for set in "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
             "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    echo "== ubench_bs pmc $i"
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/bs_pmc_$i -o run --output-format csv -- ./scripts/bitslice/ubench_bs > $OUT/bs_pmc_$i.log 2>&1 || { echo "   FAILED"; exit 1; }
  done
fi
echo done
