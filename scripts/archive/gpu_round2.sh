#!/bin/bash
# Round-2 GPU session: parity tests, smoke, bench lines (c3 with parity sample
# and CPU baselines, c2, c5, optional c4 piece plan); every step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -2 $OUT/$name.log | cut -c1-600; return $rc; }
if [ -z "$NOTESTS" ]; then
  step gpu_tests 700 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
  step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
if [ -z "$NOBENCH" ]; then
  step bench_c3 400 python -u bench.py --steps ${STEPS:-5} --warmup 1 ${BENCHARGS} || exit 1
  step bench_c2 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit 1
  step bench_c5 300 python -u bench.py --config c5 --steps 20 --warmup 2 || exit 1
fi
if [ -n "$C4" ]; then
  step bench_c4 600 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline || exit 1
fi
if [ -n "$PROFILE" ]; then
  step rocprof_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
fi
echo done
