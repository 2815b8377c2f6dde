#!/bin/bash
# Round 5: quad CFB-8 step with rounds 1-2 off the chain (hb_quad_cfb8_step2):
# PRF / prove parity tests, A/B of configs[4] against the previous build
# (HB_LIB_PATH=scripts/ab/libhb_place.so: placement only), alternating, 4
# rounds, and a kernel-trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5m}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step prove_tests 600 python -u -m pytest tests/test_gpu_quad.py tests/test_gpu_wsum.py tests/test_gpu_primes.py tests/test_gpu_configs4.py tests/test_gpu_parity.py -k "prove or quad or wsum or prime or verify or configs4 or index or prf or kat" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for r in 1 2 3 4; do
  step c5_pre_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
  HB_LIB_PATH=scripts/ab/libhb_place.so step c5_place_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
done
step stats_c5_pre 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_c5_pre -o run --output-format csv -- python3 bench.py --config c5 --steps 50 --warmup 5 --no-cpu-baseline || exit 1
echo done
