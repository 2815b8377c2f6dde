#!/bin/bash
# Round 6: conflict-free wmac slice stores -- parity, rates, LDS PMC.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6n}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -5 $OUT/$name.log | cut -c1-250; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_cxx.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step rate 300 python -u scripts/encode_rate.py 1024:10:8:cxx 1024:10:8 512:16:8 2048:4:8 1024:10:8 || exit 1
HB_ENABLE_TEST_SWITCHES=1 HB_WIDE_SYNC_ALPHA=1 step rate_sync 300 python -u scripts/encode_rate.py 1024:10:8:cxx 1024:10:8 512:16:8 2048:4:8 1024:10:8 || exit 1
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8:cxx 1024:10:8 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_lds -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:2:cxx > $OUT/pmc_lds.log 2>&1 || exit 1
echo done
