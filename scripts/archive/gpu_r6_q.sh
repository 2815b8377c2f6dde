#!/bin/bash
# Round 6: queue refill size ($HB_QCHUNK) A/B for the encode engines --
# parity at a small refill, then rates at 64 / 128 / 256 jobs per refill.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6q}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -6 $OUT/$name.log | cut -c1-250; return $rc; }
export HB_ENABLE_TEST_SWITCHES=1
HB_QCHUNK=64 step tests64 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
R="1024:10:8 512:16:8 2048:4:8 1024:10:8:cxx P256:16:16"
for k in 1 2; do
  for q in 256 128 64; do
    HB_QCHUNK=$q step rate_q${q}_$k 300 python -u scripts/encode_rate.py $R || exit 1
  done
done
echo done
