#!/bin/bash
# Round 4 final-tree check: GPU tests, smoke, and the bench lines of every
# BASELINE config (c3 default with CPU rows, c2, c4 on one GPU, c5 with CPU
# rows, the host path), each step under its own limit, stopping at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4final}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_c3 600 python -u bench.py || exit 1
step bench_c2 300 python -u bench.py --config c2 || exit 1
step bench_c4 400 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
step bench_c4_nowarmup 400 python -u bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample || exit 1
step bench_c5 300 python -u bench.py --config c5 || exit 1
step bench_host 600 python -u bench.py --host-path --steps 3 --no-cpu-baseline || exit 1
echo done
