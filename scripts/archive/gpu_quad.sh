#!/bin/bash
# Quad-engine session: GPU tests (incl. tests/test_gpu_quad.py), prove bench
# (configs[4]) with the quad engine and with HB_NO_QUAD=1, then the c3 A/B of
# experiment builds (gpu_ab.sh conventions).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-quad}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-400; return $rc; }
step gpu_tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
step c5_quad 200 python -u bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
HB_NO_QUAD=1 step c5_lane 200 python -u bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
step rocprof_c5 200 rocprofv3 --kernel-trace --stats -d $OUT/rocprof_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
for round in 1 2; do
  for v in ${VARIANTS:-base}; do
    if [ "$v" = base ]; then unset HB_LIB_PATH; else export HB_LIB_PATH=$PWD/exp_$v.so; fi
    step c3_${v}_$round 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample || exit 1
  done
done
echo done
