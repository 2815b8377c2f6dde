#!/bin/bash
# Round 5, first call: the configs[4]-width prove tests on the round-4 build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs4.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/gpu_tests_c4w.log 2>&1
rc=$?; tail -5 $OUT/gpu_tests_c4w.log; exit $rc
