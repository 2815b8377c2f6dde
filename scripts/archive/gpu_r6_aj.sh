#!/bin/bash
# Round 6: HBM traffic of the 1024-bit split encode's kernels (FETCH_SIZE,
# WRITE_SIZE in separate --pmc passes) for the wide row's roofline notes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6aj}
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 > $OUT/fetch.log 2>&1 || { echo "fetch rc=$?"; tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 > $OUT/write.log 2>&1 || { echo "write rc=$?"; tail -5 $OUT/write.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for c in ("fetch", "write"):
    agg = collections.defaultdict(list)
    for f in glob.glob(sys.argv[1] + "/" + c + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "encode" in k or "wmac" in k or "prefix" in k:
            print(c, k, "calls", len(v), "KB per call (last)", v[-1])
PY
echo done
