#!/bin/bash
# Round 6: hb_wmac_kernel with the finish's F and tags staged through LDS
# (coalesced) -- parity, rates, kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6u}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -6 $OUT/$name.log | cut -c1-250; return $rc; }
step tests 500 python -u -m pytest ${TESTS:-tests/test_gpu_wide.py tests/test_gpu_cxx.py tests/test_gpu_parity.py} -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
R="${R:-1024:10:8 512:16:8 2048:4:8 1024:10:8:cxx}"
step rate_1 300 python -u scripts/encode_rate.py $R || exit 1
step rate_2 300 python -u scripts/encode_rate.py $R || exit 1
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 scripts/encode_rate.py $R || exit 1
python3 - $OUT/stats <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wmac" in r["Name"] or "encode" in r["Name"]:
            print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
echo done
