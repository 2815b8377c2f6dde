#!/bin/bash
# Round 6: the mid-size path with the MFMA MAC -- parity (small/mid/wide
# tests), then mid vs two-pass sweeps at 512/1024/2048 bits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6j}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; cat $OUT/$name.log | tail -14 | cut -c1-200; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py tests/test_gpu_surface.py tests/test_gpu_primes.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
SIZES="1024:10:0.1 1024:10:0.25 1024:10:0.5 1024:10:1 1024:10:2 1024:10:2.6 512:16:0.25 512:16:0.5 512:16:1 512:16:1.2 2048:4:0.1 2048:4:0.25 2048:4:1"
step mid 300 python -u scripts/encode_rate.py $SIZES || exit 1
HB_ENABLE_TEST_SWITCHES=1 HB_MID_BLOCKS=0 step twopass 300 python -u scripts/encode_rate.py $SIZES || exit 1
echo done
