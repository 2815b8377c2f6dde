#!/bin/bash
# A/B experiment session: bench variants (HB_LIB_PATH) and PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-exp}
mkdir -p $OUT
run() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"frac": [0-9.]*' $OUT/$name.log | tr '\n' ' '; echo; return $rc; }
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then unset HB_LIB_PATH; else export HB_LIB_PATH=$PWD/exp_$v.so; fi
  run c3_$v 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  [ -n "$C2" ] && { run c2_$v 200 python -u bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline || exit 1; }
done
unset HB_LIB_PATH
if [ -n "$PMC" ]; then
  for ctr in $PMC; do
    run pmc_$ctr 300 rocprofv3 --pmc $ctr -d $OUT/pmc_$ctr -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline || exit 1
  done
fi
echo done
