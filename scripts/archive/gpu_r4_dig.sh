#!/bin/bash
# Round 4: retry-list digests (HB_RETRY_DIGEST, exp_dg1.so) against the same
# code without them (exp_dg0.so) and the in-tree build: parity subsets on both
# variant builds, then a same-box A/B at configs[2] (c3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r4n}
mkdir -p $OUT
K="(golden_device_path or device_resident_64mib or mfma_mac or two_pass or async or repeated or shards or generic or sectors_short) and not prepare"
for v in dg1 dg0; do
  echo "== parity $v"
  HB_LIB_PATH=./exp_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/parity_$v.log 2>&1 || { tail -30 $OUT/parity_$v.log; exit 1; }
  tail -n 1 $OUT/parity_$v.log
done
TAG=${TAG:-r4n}/c3 ROUNDS=${ROUNDS:-4} PARITY=1 VARIANTS="base dg0:HB_LIB_PATH=./exp_dg0.so dg1:HB_LIB_PATH=./exp_dg1.so" bash scripts/gpu_r4.sh || exit 1
echo all done
