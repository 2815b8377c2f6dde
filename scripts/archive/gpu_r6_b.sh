#!/bin/bash
# Round 6: the split wide-prime encode (F-only PRF passes + MFMA MAC) --
# parity tests, rates at 512/1024/2048 bits, kernel split, then the full
# default bench line (wide + configs1 rows).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6b}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -3 $OUT/$name.log | cut -c1-400; return $rc; }
step wide_tests 400 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs4.py::test_configs1_host_gather_prove_at_26_bit_index_width -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step rate_wide 300 python -u scripts/encode_rate.py 1024:10:8 512:16:8 2048:4:8 || exit 1
step stats_wide 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_wide -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 || exit 1
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step bench 600 python -u bench.py || exit 1
echo done
