#!/bin/bash
# Round 6: host-memory encode rates at 256 and 1024 bits (raw and API), and
# with the mid-size path off (HB_MID_BLOCKS=1: two-pass per 256 MiB chunk).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6s}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -4 $OUT/$name.log | cut -c1-400; return $rc; }
step host 400 python -u scripts/host_rate.py 4 || exit 1
export HB_ENABLE_TEST_SWITCHES=1
HB_MID_BLOCKS=1 step host_nomid 400 python -u scripts/host_rate.py 4 || exit 1
step rate_256m 200 python -u scripts/encode_rate.py 1024:10:0.25 1024:10:1 P256:16:0.25 || exit 1
HB_MID_BLOCKS=1 step rate_256m_nomid 200 python -u scripts/encode_rate.py 1024:10:0.25 1024:10:1 P256:16:0.25 || exit 1
echo done
