#!/bin/bash
# Round 6: the cxx prf's 1024-bit F-only kernel in 768-thread workgroups --
# parity, rates, kernel stats and register / scratch use.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6ai}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -3 $OUT/$name.log | cut -c1-250; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_cxx.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step rate_1 300 python -u scripts/encode_rate.py 1024:10:8:cxx 1024:10:8:cxx 2048:4:8:cxx 512:16:8:cxx || exit 1
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8:cxx || exit 1
python3 - $OUT/stats <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wmac" in r["Name"] or "encode" in r["Name"]:
            print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
for f in glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        if "encode" in r["Kernel_Name"] and r["Kernel_Name"] not in seen:
            seen.add(r["Kernel_Name"])
            print("  res", r["Kernel_Name"][:50], {k: v for k, v in r.items() if "GPR" in k or "Scratch" in k or "Workgroup_Size_X" in k})
PY
echo done
