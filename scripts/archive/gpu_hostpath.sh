#!/bin/bash
# Host-path rates (pinned / pageable / drop-in API BytesIO and mmap'd file) and
# a rehearsal of bench.py's self-spawned N-rank path with both ranks on the
# box's one GPU (HB_BENCH_SAME_DEVICE=1, 16 GiB per rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-hostpath}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-300; return $rc; }
step host_path 400 python -u bench.py --host-path --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
HB_BENCH_SAME_DEVICE=1 step ranks2_c3 300 python -u bench.py --gpus 2 --gib 16 --steps 3 --warmup 1 --no-cpu-baseline || exit 1
HB_BENCH_SAME_DEVICE=1 step ranks2_c4 300 python -u bench.py --gpus 2 --config c4 --gib 16 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
echo done
