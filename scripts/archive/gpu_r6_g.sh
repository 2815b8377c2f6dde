#!/bin/bash
# Round 6: wmac shape A/B -- 8 waves x 256 blocks (in-tree) vs 4 waves x 128
# blocks (exp_ng8.so); parity of the in-tree build first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6g}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -4 $OUT/$name.log | cut -c1-300; return $rc; }
step wide_tests 400 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for v in new old new old; do
  if [ $v = old ]; then export HB_LIB_PATH=$PWD/exp_ng8.so; else unset HB_LIB_PATH; fi
  step rate_$v 200 python -u scripts/encode_rate.py 1024:10:8 512:16:8 2048:4:8 || exit 1
done
unset HB_LIB_PATH
step stats_new 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_new -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 512:16:8 2048:4:8 || exit 1
echo done
