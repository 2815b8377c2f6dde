#!/bin/bash
# Round 4 session script: optional GPU tests, then an A/B of bench c3 over
# variants given as environment assignments ("name:VAR=val,VAR2=val" or
# "name" for the plain build; HB_LIB_PATH=<so> selects an experiment build),
# rounds alternating, then optional PMC passes (COUNTERS, ';'-separated sets)
# per variant in PMCVARIANTS, then optional rocprof stats of the plain build.
# Every step runs under its own time limit; the script stops at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-400; return $rc; }
# apply a variant spec: exports its assignments in the current shell
APPLIED=""
apply() {
  local spec=$1 kv
  for kv in $APPLIED; do unset "$kv"; done
  APPLIED=""
  VNAME=${spec%%:*}
  if [ "$spec" != "$VNAME" ]; then
    IFS=',' read -ra KVS <<< "${spec#*:}"
    for kv in "${KVS[@]}"; do export "$kv"; APPLIED="$APPLIED ${kv%%=*}"; done
  fi
}
if [ -n "$TESTS" ]; then
  step gpu_tests ${TESTLIMIT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
fi
if [ -n "$SMOKE" ]; then
  step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
for round in $(seq ${ROUNDS:-0}); do
  for spec in ${VARIANTS:-base}; do
    apply "$spec"
    ps="--no-parity-sample"; [ -n "$PARITY" ] && [ $round = 1 ] && ps=""
    step c3_${VNAME}_$round 300 python -u bench.py --steps ${STEPS:-10} --warmup 1 --no-cpu-baseline $ps ${BENCHARGS} || exit 1
  done
done
apply base
IFS=';' read -ra SETS <<< "$COUNTERS"
for spec in ${PMCVARIANTS:-base}; do
  apply "$spec"
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    echo "== pmc $VNAME $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_${VNAME}_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample ${BENCHARGS} > $OUT/pmc_${VNAME}_$i.log 2>&1 || { echo "   pmc FAILED"; exit 1; }
  done
done
apply base
if [ -n "$STATS" ]; then
  for spec in $STATS; do
    apply "$spec"
    step stats_${VNAME} 400 rocprofv3 --kernel-trace --stats -d $OUT/stats_${VNAME} -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample ${BENCHARGS} || exit 1
  done
fi
if [ -n "$COLD" ]; then
  apply base
  HB_TRACE_PHASES=1 step c4_cold_trace 300 python3 -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample || exit 1
  HB_TRACE_PHASES=1 step c3_cold_trace 300 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample || exit 1
fi
if [ -n "$FULLBENCH" ]; then
  apply base
  step bench_full 600 python -u bench.py ${FULLBENCH_ARGS} || exit 1
fi
echo done
