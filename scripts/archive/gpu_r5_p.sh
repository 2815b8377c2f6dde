#!/bin/bash
# Round 5: the fused prove's host polls its completion token in the coherent
# pinned buffer (finish_sums): fused + prove tests, A/B of configs[4] against
# HB_SYNC_WAIT (hipStreamSynchronize), alternating, 4 rounds; verify timed in
# the same lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5p}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step prove_tests 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_quad.py tests/test_gpu_wsum.py tests/test_gpu_primes.py tests/test_gpu_configs4.py tests/test_gpu_parity.py -k "fused or prove or quad or wsum or prime or verify or configs4 or index or prf or kat or queue" -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
export HB_ENABLE_TEST_SWITCHES=1
for r in 1 2 3 4; do
  step c5_poll_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
  HB_SYNC_WAIT=1 step c5_sync_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1
done
echo done
