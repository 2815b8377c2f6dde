#!/bin/bash
# Round 4: weighted-sum kernel with the status word closed by workgroup (0, 0)
# and a shorter final tree (exp_ws.so): the whole GPU suite on the variant,
# then a same-box A/B of the configs[4] prove.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r4q}
mkdir -p $OUT
echo "== gpu tests on exp_ws.so"
HB_LIB_PATH=./exp_ws.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $OUT/gpu_tests_ws.log 2>&1 || { tail -30 $OUT/gpu_tests_ws.log; exit 1; }
tail -n 1 $OUT/gpu_tests_ws.log
TAG=${TAG:-r4q}/c5 ROUNDS=${ROUNDS:-4} STEPS=200 BENCHARGS="--config c5" VARIANTS="base ws:HB_LIB_PATH=./exp_ws.so" bash scripts/gpu_r4.sh || exit 1
echo all done
