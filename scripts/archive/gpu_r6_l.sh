#!/bin/bash
# Round 6: the split MAC for the cxx prf -- parity (wide + cxx test files),
# then the cxx 1024-bit rate and its kernel split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6l}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -4 $OUT/$name.log | cut -c1-250; return $rc; }
step tests 500 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_cxx.py tests/test_gpu_swizzle.py tests/test_gpu_surface.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step rate 300 python -u scripts/encode_rate.py 1024:10:8:cxx 1024:10:8:cxx P256:16:8:cxx 1024:10:8 || exit 1
step stats 300 rocprofv3 --kernel-trace --stats -d $OUT/stats -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8:cxx || exit 1
echo done
