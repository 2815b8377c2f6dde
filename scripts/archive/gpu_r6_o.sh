#!/bin/bash
# Round 6: the overlapped MAC (F-free half beside the PRF passes + combine) --
# parity, then A/B against the one-kernel MAC after the passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6o}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -6 $OUT/$name.log | cut -c1-250; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_cxx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
R="1024:10:8:cxx 1024:10:8 512:16:8 2048:4:8"
export HB_ENABLE_TEST_SWITCHES=1
for k in 1 2; do
  step rate_ov_$k 300 python -u scripts/encode_rate.py $R || exit 1
  HB_WIDE_NO_OVERLAP=1 step rate_seq_$k 300 python -u scripts/encode_rate.py $R || exit 1
done
HB_WMAC_WPE=4 step rate_ov_wpe4 300 python -u scripts/encode_rate.py $R || exit 1
HB_WMAC_WPE=3 step rate_ov_wpe3 300 python -u scripts/encode_rate.py $R || exit 1
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8:cxx 1024:10:8 || exit 1
echo done
