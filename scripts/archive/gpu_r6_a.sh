#!/bin/bash
# Round 6, first lease: the new GPU tests (import surface, alpha position
# limit, token word), the whole GPU suite, smoke, and the kernel split of the
# 1024-bit S = 10 encode (PySwizzle's defaults) before the wide-prime work.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6a}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -3 $OUT/$name.log | cut -c1-300; return $rc; }
step new_tests 300 python -u -m pytest tests/test_gpu_surface.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
step rate_wide 300 python -u scripts/encode_rate.py 1024:10:8 512:16:8 P256:16:8 || exit 1
step stats_wide 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_wide -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 || exit 1
echo done
