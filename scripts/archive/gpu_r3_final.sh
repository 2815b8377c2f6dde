#!/bin/bash
# Round-3 evidence, part 1: GPU parity tests, smoke, the default bench line
# (c3 with CPU rows and parity sample), c2 and c5 lines, rocprofv3 stats of c3.
# Part 2 (PART=2): host-path bench and PMC passes.  Every step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3final}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -n 2 $OUT/$name.log | cut -c1-400; return $rc; }
if [ "${PART:-1}" = 1 ]; then
  step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
  step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
  step bench_c3 300 python -u bench.py || exit 1
  step bench_c2 200 python -u bench.py --config c2 --steps 10 --warmup 2 || exit 1
  step bench_c5 200 python -u bench.py --config c5 --steps 20 --warmup 2 || exit 1
  step rocprof_c3 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
else
  step bench_host 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample --host-path || exit 1
  i=0
  for set in "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAVES" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    echo "== pmc pass $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample > $OUT/pmc_$i.log 2>&1 || { echo "   FAILED"; exit 1; }
  done
fi
echo done
