#!/bin/bash
# One GPU session: parity tests, smoke, bench (c3 + c2), optional A/B and
# rocprofv3 kernel trace.  Every GPU step has its own time limit; the script
# stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -3 $OUT/$name.log; return $rc; }
if [ -z "$NOTESTS" ]; then
  step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
  step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
fi
step bench_c3 400 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 10 ${HOSTPATH:+--host-path} || exit 1
step bench_c2 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit 1
if [ -n "$PROVE" ]; then
  step bench_c5 300 python -u bench.py --config c5 --steps 20 --warmup 2 || exit 1
fi
if [ -n "$AB" ]; then
  step bench_c3_single 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --single-pass || exit 1
  step bench_c2_single 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline --single-pass || exit 1
fi
if [ -n "$PROFILE" ]; then
  step rocprof_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
fi
echo done
