#!/bin/bash
# Round 6: where the split two-pass encode overtakes the mid-size quad-PRF
# path for wide primes (1024-bit S = 10, 512-bit S = 16): default vs
# HB_MID_BLOCKS=0 (two-pass above the placed-wave limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6i}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; cat $OUT/$name.log | cut -c1-200; return $rc; }
SIZES="1024:10:0.1 1024:10:0.25 1024:10:0.5 1024:10:1 1024:10:2 1024:10:2.6 512:16:0.25 512:16:0.5 512:16:1 512:16:1.2 2048:4:0.25 2048:4:1"
step mid 300 python -u scripts/encode_rate.py $SIZES || exit 1
HB_ENABLE_TEST_SWITCHES=1 HB_MID_BLOCKS=0 step twopass 300 python -u scripts/encode_rate.py $SIZES || exit 1
echo done
