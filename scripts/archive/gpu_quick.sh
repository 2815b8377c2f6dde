#!/bin/bash
# Quick GPU iteration: selected tests, bench c3 (+variants), optional rocprof of c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quick}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -2 $OUT/$name.log | cut -c1-400; return $rc; }
if [ -n "$TESTS" ]; then
  step gpu_tests 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
fi
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset HB_LIB_PATH; else export HB_LIB_PATH=$PWD/exp_$v.so; fi
  step c3_$v 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCHARGS} || exit 1
done
unset HB_LIB_PATH
if [ -n "$PROFC5" ]; then
  step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
fi
if [ -n "$PROFC3" ]; then
  step rocprof_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
fi
echo done
