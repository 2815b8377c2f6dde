#!/bin/bash
# Round 5: full tree check -- GPU suite, smoke, default bench (sustained +
# host_path rows), c2, c5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5e}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
step gpu_tests 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step bench_c3 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step bench_c2 300 python -u bench.py --config c2 || exit 1
step bench_c5 300 python -u bench.py --config c5 || exit 1
echo done
