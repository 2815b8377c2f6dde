#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter set,
# each under its own kill timeout).  COUNTERS: ';'-separated sets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p $OUT
if [ -n "$LIST" ]; then timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"; fi
IFS=';' read -ra SETS <<< "$COUNTERS"
i=0
for mode in ${MODES:-two single}; do
  extra=""; [ "$mode" = single ] && extra="--single-pass"; [ "$mode" = cxx ] && extra="--prf cxx"
  for set in "${SETS[@]}"; do
    i=$((i+1))
    echo "== pass $i ($mode): $set"
    timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/p${i}_$mode -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --gib ${GIB:-8} $extra > $OUT/p${i}_$mode.log 2>&1
    rc=$?; echo "   rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p${i}_$mode.log; exit 1; }
  done
done
echo done
