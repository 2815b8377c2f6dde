#!/bin/bash
# GPU tests, then the host-path rates with the pinned bounce staging and
# without it (HB_NO_BOUNCE=1: the runtime's own pageable staging).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-bounce}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-200; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step host_bounce 400 python -u bench.py --host-path --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
HB_NO_BOUNCE=1 step host_nobounce 400 python -u bench.py --host-path --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
HB_COPY_THREADS=8 step host_bounce8 400 python -u bench.py --host-path --steps 2 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
echo done
