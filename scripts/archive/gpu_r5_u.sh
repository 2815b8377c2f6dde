#!/bin/bash
# Round 5: small-input encode path (placed quad PRF + hb_mac_kernel; quad
# PRF launches placed by SIMD): the whole GPU suite, the drop-in API's
# small-input latencies against HB_NO_SMALL_ENCODE (+ HB_NO_PROVE_PLACE for the
# unplaced quad PRF launches), alternating, and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5u}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
export HB_ENABLE_TEST_SWITCHES=1
for r in 1 2; do
  step api_small_$r 300 python -u scripts/api_latency.py || exit 1
  HB_NO_SMALL_ENCODE=1 HB_NO_PROVE_PLACE=1 step api_twopass_$r 300 python -u scripts/api_latency.py || exit 1
done
unset HB_ENABLE_TEST_SWITCHES
step bench_c3 600 python -u bench.py || exit 1
echo done
