#!/bin/bash
# Round 6: what binds hb_wmac_kernel -- its time with the B (file) loads, the
# A-fragment loads or the MFMAs taken out (HB_WMAC_EXP, results invalid).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6t}
mkdir -p $OUT
export HB_ENABLE_TEST_SWITCHES=1
for e in ${EXPS:-0 1 2 4 3 5 6 7}; do
  echo "== exp $e"
  HB_WMAC_EXP=$e timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/e$e -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8 512:16:8 > $OUT/e$e.log 2>&1 || { echo "rc=$?"; tail -5 $OUT/e$e.log; exit 1; }
  python3 - $OUT/e$e <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "wmac" in r["Name"]:
            print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
for f in glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        if "wmac" in r["Kernel_Name"] and r["Kernel_Name"] not in seen:
            seen.add(r["Kernel_Name"])
            print("  vgpr", {k: v for k, v in r.items() if "GPR" in k or "LDS" in k or "Scratch" in k})
PY
done
echo done
