#!/bin/bash
# Round 4: is hb_wsum_kernel's 0.04 ms a translation cost?  Kernel stats of
# the configs[4] prove (10,000 random indices) on a 64 GiB file against the
# same prove on 1 GiB and 8 GiB files (same index count, fewer pages).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4o}
mkdir -p $OUT
for g in 64 8 1; do
  echo "== c5 ${g} GiB"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c5_$g -o run --output-format csv -- \
    python3 bench.py --config c5 --gib $g --steps 50 --warmup 5 --no-cpu-baseline --no-parity-sample > $OUT/c5_$g.log 2>&1 || { tail -20 $OUT/c5_$g.log; exit 1; }
  grep '^{' $OUT/c5_$g.log | cut -c1-300
done
echo all done
