#!/bin/bash
# Round 4: the MFMA-table/prefix overlap (exp_ovl.so) and the MFMA MAC at
# S = 1 (HB_MFMA_MIN_S=1 on the same build): parity subsets on the variant
# build, then same-box A/Bs at configs[2] (c3) and configs[1] (c2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r4l}
mkdir -p $OUT
K="(golden_device_path or device_resident_64mib or mfma_mac or two_pass or async or repeated or shards) and not prepare"
echo "== parity ovl"
HB_LIB_PATH=./exp_ovl.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/parity_ovl.log 2>&1 || { tail -30 $OUT/parity_ovl.log; exit 1; }
tail -1 $OUT/parity_ovl.log
echo "== parity ovl min_s=1"
HB_LIB_PATH=./exp_ovl.so HB_MFMA_MIN_S=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -k "$K" > $OUT/parity_mins1.log 2>&1 || { tail -30 $OUT/parity_mins1.log; exit 1; }
tail -1 $OUT/parity_mins1.log
TAG=${TAG:-r4l}/c3 ROUNDS=${ROUNDS:-4} VARIANTS="base ovl:HB_LIB_PATH=./exp_ovl.so" bash scripts/gpu_r4.sh || exit 1
TAG=${TAG:-r4l}/c2 ROUNDS=${ROUNDS:-4} BENCHARGS="--config c2" \
  VARIANTS="base ovl:HB_LIB_PATH=./exp_ovl.so mins1:HB_LIB_PATH=./exp_ovl.so,HB_MFMA_MIN_S=1" bash scripts/gpu_r4.sh || exit 1
echo all done
