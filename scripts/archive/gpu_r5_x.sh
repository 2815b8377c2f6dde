#!/bin/bash
# Round 5: small-input encode with F and alpha in one launch, no page-locking
# under 32 MiB: the whole GPU suite, the API small-input latencies, and
# small-input latencies (A/B), and the default bench line (its host-file
# prove row uploads the 4 GiB file).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5x}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
export HB_ENABLE_TEST_SWITCHES=1
for r in 1 2; do
  step api_new_$r 300 python -u scripts/api_latency.py || exit 1
  HB_NO_SMALL_ENCODE=1 step api_twopass_$r 300 python -u scripts/api_latency.py || exit 1
done
unset HB_ENABLE_TEST_SWITCHES
step bench_c3 600 python -u bench.py || exit 1
echo done
