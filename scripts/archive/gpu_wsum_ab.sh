#!/bin/bash
# A/B of the weighted-sum grid (HB_WSUM_TPT terms per thread) on configs[4]
# under rocprofv3 kernel stats, plus the host-path / API rates.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-wsum}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
for t in 1 4 16 40; do
  HB_WSUM_TPT=$t step c5_tpt$t 200 rocprofv3 --kernel-trace --stats -d $OUT/prof_tpt$t -o run --output-format csv -- python3 bench.py --config c5 --gib 8 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
done
step host_path 400 python -u bench.py --host-path --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
echo done
