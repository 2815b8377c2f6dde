#!/bin/bash
# Round 5 final-tree check: GPU tests, smoke, the bench lines of every
# BASELINE config (c3 with the driver's own arguments), rocprof stats and the
# PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) of c3.  Each step under its own
# limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5final}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
step gpu_tests 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_c3 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step bench_c2 300 python -u bench.py --config c2 || exit 1
step bench_c4 400 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
step bench_c5 300 python -u bench.py --config c5 || exit 1
step stats_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/stats_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample --no-host-path --sustain-seconds 0 || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample --no-host-path --sustain-seconds 0 > $OUT/pmc_$i.log 2>&1 || { echo "   pmc FAILED"; exit 1; }
done
step stats_c5 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
echo done
