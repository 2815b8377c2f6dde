#!/bin/bash
# cxx two-pass (MFMA MAC) session: GPU tests, then configs[2] in cxx mode
# two-pass vs single-pass, the PySwizzle headline, and a rocprof summary.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cxx2}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-250; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step c3_cxx 300 python -u bench.py --prf cxx --steps 5 --warmup 1 --no-cpu-baseline || exit 1
step c3_cxx_single 300 python -u bench.py --prf cxx --single-pass --steps 5 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
step c3 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit 1
step rocprof_c3_cxx 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3_cxx -o run --output-format csv -- python3 bench.py --prf cxx --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
echo done
