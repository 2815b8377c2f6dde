#!/bin/bash
# cxx-prf session: GPU tests, cxx benches, kernel-trace profiles of both modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cxx}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -3 $OUT/$name.log | cut -c1-1500; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step bench_c3_cxx 300 python -u bench.py --prf cxx --steps 5 --warmup 1 --cpu-seconds 10 || exit 1
step bench_c2_cxx 200 python -u bench.py --prf cxx --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit 1
step rocprof_c3 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
step rocprof_c3_cxx 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3_cxx -o run --output-format csv -- python3 bench.py --prf cxx --steps 3 --warmup 1 --no-cpu-baseline || exit 1
echo done
