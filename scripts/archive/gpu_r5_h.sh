#!/bin/bash
# Round 5: the prove's device gather (hb_gather_block in the PRF kernel, wsum
# over the compact buffer): GPU suite, then a same-box A/B of configs[4]
# against HB_NO_PROVE_GATHER (the file-gathering sum), alternating, 4 rounds,
# and rocprof kernel stats of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5h}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step gpu_tests 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
export HB_ENABLE_TEST_SWITCHES=1
for r in 1 2 3 4; do
  step c5_gather_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
  HB_NO_PROVE_GATHER=1 step c5_file_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
done
step stats_c5_gather 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c5_gather -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
HB_NO_PROVE_GATHER=1 step stats_c5_file 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c5_file -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
echo done
