#!/bin/bash
# A/B on one box: optional GPU tests, then bench c3 alternating the in-tree
# build ("base") and experiment builds exp_<v>.so (HB_LIB_PATH), then optional
# PMC passes (COUNTERS, ';'-separated sets) on the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
if [ -n "$TESTS" ]; then
  step gpu_tests 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
fi
r=0
for round in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS:-base}; do
    r=$((r+1))
    if [ "$v" = base ]; then unset HB_LIB_PATH; else export HB_LIB_PATH=$PWD/exp_$v.so; fi
    ps="--no-parity-sample"; [ -n "$PARITY" ] && [ $round = 1 ] && ps=""
    step c3_${v}_$round 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline $ps ${BENCHARGS} || exit 1
  done
done
unset HB_LIB_PATH
IFS=';' read -ra SETS <<< "$COUNTERS"
for v in ${PMCVARIANTS:-base}; do
  if [ "$v" = base ]; then unset HB_LIB_PATH; else export HB_LIB_PATH=$PWD/exp_$v.so; fi
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    echo "== pmc $v $i: $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_${v}_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample ${BENCHARGS} > $OUT/pmc_${v}_$i.log 2>&1 || { echo "   pmc FAILED"; exit 1; }
  done
done
unset HB_LIB_PATH
echo done
