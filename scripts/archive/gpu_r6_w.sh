#!/bin/bash
# Round 6: hb_wmac_kernel<64> waves-per-SIMD bound A/B (HB_WMAC_WPE) at 2048 bits.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6w}
mkdir -p $OUT
export HB_ENABLE_TEST_SWITCHES=1
for w in 1 3 4 1 3; do
  echo "== wpe $w"
  HB_WMAC_WPE=$w timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/w$w -o run --output-format csv -- python3 scripts/encode_rate.py 2048:4:8 > $OUT/w$w.log 2>&1 || { echo "rc=$?"; tail -5 $OUT/w$w.log; exit 1; }
  grep prime_bits $OUT/w$w.log
  python3 - $OUT/w$w <<'PY'
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
            print("  res", {k: v for k, v in r.items() if "GPR" in k or "LDS" in k or "Scratch" in k})
PY
done
echo done
