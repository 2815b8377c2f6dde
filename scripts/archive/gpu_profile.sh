#!/bin/bash
# Profiles for the committed numbers: rocprofv3 kernel-trace stats of the c3 /
# c2 / c5 bench runs and PMC passes (one counter set per run) on c3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; return $rc; }
step rocprof_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
step rocprof_c2 200 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c2 -o run --output-format csv -- python3 bench.py --config c2 --steps 5 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
step rocprof_c5 200 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
i=0
IFS=';' read -ra SETS <<< "${PMC:-FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES}"
for set in "${SETS[@]}"; do
  i=$((i+1))
  echo "== pmc $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample > $OUT/pmc_$i.log 2>&1 || { echo "   pmc FAILED"; exit 1; }
done
echo done
