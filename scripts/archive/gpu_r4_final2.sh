#!/bin/bash
# Round 4 final-tree check of the current build (16x16x64 MAC, plain finish):
# GPU tests, smoke, the bench lines of every BASELINE config, rocprof stats
# and PMC passes (FETCH_SIZE / WRITE_SIZE / SQ) of c3.  Each step under its
# own limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4final2}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_c3 600 python -u bench.py || exit 1
step bench_c2 300 python -u bench.py --config c2 || exit 1
step bench_c4 400 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
step bench_c4_nowarmup 400 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample || exit 1
step bench_c5 300 python -u bench.py --config c5 || exit 1
step stats_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/stats_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc $i: $set"
  timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample > $OUT/pmc_$i.log 2>&1 || { echo "   pmc FAILED"; exit 1; }
done
echo done
