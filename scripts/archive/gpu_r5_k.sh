#!/bin/bash
# Round 5: prime sizes 129-2048 bits (every limb count) and KeyedPRF ranges
# vs the oracle; the GPU suite; configs[4] without the prove's timing events.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5k}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step primes 600 python -u -m pytest tests/test_gpu_primes.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step gpu_tests 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
for r in 1 2; do step c5_$r 300 python -u bench.py --config c5 --steps 200 --warmup 20 --no-cpu-baseline || exit 1; done
echo done
