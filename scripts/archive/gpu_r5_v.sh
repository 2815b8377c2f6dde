#!/bin/bash
# Round 5: small host files proved device-resident after one upload
# (HB_NO_PROVE_UPLOAD: the host gather): the whole GPU suite, the API's
# small-input latencies (A/B), and the default bench line (its host-file
# prove row uploads the 4 GiB file).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5v}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
export HB_ENABLE_TEST_SWITCHES=1
for r in 1 2; do
  step api_upload_$r 300 python -u scripts/api_latency.py || exit 1
  HB_NO_PROVE_UPLOAD=1 step api_gather_$r 300 python -u scripts/api_latency.py || exit 1
done
unset HB_ENABLE_TEST_SWITCHES
step bench_c3 600 python -u bench.py || exit 1
echo done
