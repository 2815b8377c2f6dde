#!/bin/bash
# Round 5: the provenance-stamped build with the wsum completion token, the
# load-only launcher split, gated switches and HB_HOST_REGISTER: GPU tests,
# smoke, the default bench line (now with host_path), c5, rocprof stats of c3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5b}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-400; return $rc; }
step gpu_tests 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_c3 600 python -u bench.py || exit 1
step bench_c5 300 python -u bench.py --config c5 || exit 1
step stats_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/stats_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample --no-host-path || exit 1
echo done
