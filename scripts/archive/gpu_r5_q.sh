#!/bin/bash
# Round 5: fused verify (hb_verify_fused_kernel): its tests + the prove / PRF
# parity tests, then A/B of configs[4]'s verify time against
# HB_NO_VERIFY_FUSE (the launch sequence), alternating, 4 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5q}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step fused_tests 400 python -u -m pytest tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step prove_tests 600 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_wsum.py tests/test_gpu_primes.py tests/test_gpu_configs4.py tests/test_gpu_parity.py -k "prove or quad or wsum or prime or verify or configs4 or index or prf or kat" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
export HB_ENABLE_TEST_SWITCHES=1
for r in 1 2 3 4; do
  step c5_vfused_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
  HB_NO_VERIFY_FUSE=1 step c5_vseq_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
done
step stats_c5_vfused 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c5_vfused -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
echo done
