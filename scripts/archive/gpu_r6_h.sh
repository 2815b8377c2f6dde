#!/bin/bash
# Round 6 checkpoint: whole GPU suite, smoke, the default bench line (wide and
# configs1 rows) and its rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6h}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -2 $OUT/$name.log | cut -c1-300; return $rc; }
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench 600 python -u bench.py || exit 1
step stats_bench 400 rocprofv3 --kernel-trace --stats -d $OUT/stats_bench -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample --no-host-path --no-prove --sustain-seconds 0 || exit 1
echo done
