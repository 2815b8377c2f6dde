#!/bin/bash
# Round 6: the cxx prf's encode at its API's 1024-bit prime (and 256-bit),
# and a same-device rehearsal of the N = 2 bench path on this tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r6k}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -4 $OUT/$name.log | cut -c1-250; return $rc; }
step rate_cxx 300 python -u scripts/encode_rate.py 1024:10:8:cxx P256:16:8:cxx 1024:10:8 || exit 1
step stats_cxx 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_cxx -o run --output-format csv -- python3 scripts/encode_rate.py 1024:10:8:cxx || exit 1
HB_BENCH_SAME_DEVICE=1 step rehearsal_c4_n2 300 python -u bench.py --gpus 2 --gib 2 --steps 2 --warmup 1 || exit 1
echo done
