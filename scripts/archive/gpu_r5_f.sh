#!/bin/bash
# Round 5: host-path rows of the default bench vs the standalone probe on the same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r5f}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
df -h /tmp > $OUT/df_tmp.txt 2>&1; mount | grep -E " /tmp | / " > $OUT/mount.txt 2>&1; free -g > $OUT/free.txt 2>&1
step bench_c3 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
step probe2 300 python3 -u scripts/host_path_probe2.py || exit 1
step bench_c3_nocpu 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-parity-sample --sustain-seconds 0 || exit 1
echo done
