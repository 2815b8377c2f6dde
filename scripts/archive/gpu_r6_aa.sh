#!/bin/bash
# Round 6: mid-size path vs two-pass engine crossover for primes above 256
# bits after the 64-job refills and the coalesced MAC finish
# (HB_MID_BLOCKS=1 forces the two-pass engine).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6aa}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; cut -c1-200 $OUT/$name.log | grep prime_bits; return $rc; }
export HB_ENABLE_TEST_SWITCHES=1
R="1024:10:0.5 1024:10:1 1024:10:1.5 1024:10:2 512:16:0.5 512:16:1 512:16:2 2048:4:0.5 2048:4:1 2048:4:2"
step mid 300 python -u scripts/encode_rate.py $R || exit 1
HB_MID_BLOCKS=1 step twopass 300 python -u scripts/encode_rate.py $R || exit 1
step mid2 300 python -u scripts/encode_rate.py $R || exit 1
HB_MID_BLOCKS=1 step twopass2 300 python -u scripts/encode_rate.py $R || exit 1
echo done
