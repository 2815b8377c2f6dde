#!/bin/bash
# Fused-prove + tag-store build: GPU tests, smoke, configs[4] fused vs
# two-launch, configs[2] / configs[1] benches, rocprof kernel stats of c3 and c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fused}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-250; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 120 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_c5 300 python -u bench.py --config c5 --steps 20 --warmup 2 || exit 1
HB_NO_FUSE=1 step bench_c5_nofuse 300 python -u bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
step bench_c3 400 python -u bench.py --steps 5 --warmup 1 || exit 1
step bench_c2 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit 1
step rocprof_c3 400 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
step rocprof_c5 300 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
echo done
