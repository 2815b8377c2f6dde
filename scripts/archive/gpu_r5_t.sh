#!/bin/bash
# Round 5: small-input latency of the drop-in API, and where a 1 MiB
# PySwizzle-defaults encode (S = 10, 1024-bit) spends it (kernel trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5t}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step api_latency 300 python -u scripts/api_latency.py || exit 1
step trace_api 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_api -o run --output-format csv -- python3 scripts/api_latency.py || exit 1
echo done
