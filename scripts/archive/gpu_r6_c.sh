#!/bin/bash
# Round 6: wmac v2 (tiles split over the workgroup's waves) -- parity, then
# the 1024-bit rate with the MAC kernel's waves-per-SIMD bound A/B'd, kernel split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6c}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -4 $OUT/$name.log | cut -c1-300; return $rc; }
step wide_tests 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_surface.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for wpe in 3 3; do
  HB_ENABLE_TEST_SWITCHES=1 HB_WMAC_WPE=$wpe step rate_wpe$wpe 200 python -u scripts/encode_rate.py 1024:10:8 512:16:8 2048:4:8 || exit 1
done
step stats_wide 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_wide -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 512:16:8 2048:4:8 || exit 1
echo done
