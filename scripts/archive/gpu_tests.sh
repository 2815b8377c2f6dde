#!/bin/bash
# GPU parity tests (+ optional microbench) in one call; every step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tests}
mkdir -p $OUT
if [ -n "$UBENCH" ]; then timeout -k 10 120 ./scripts/ubench_int > $OUT/ubench_int.txt 2>&1 || exit 1; fi
timeout -k 10 ${LIMIT:-700} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests.log 2>&1
rc=$?; tail -5 $OUT/gpu_tests.log; exit $rc
