#!/bin/bash
# A/B of library variants on configs[2] (+ optional PMC passes on one variant).
#   VARIANTS="late early base"  (exp_<v>.so; base = in-tree); a variant "v:ENV=1" sets ENV for that run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for spec in ${VARIANTS:-base}; do
  v=${spec%%:*}; envs=""; [ "$spec" != "$v" ] && envs=${spec#*:}
  lib=""; [ "$v" != base ] && lib=$PWD/exp_$v.so
  name=c3_${v}${envs:+_$(echo $envs | tr '=' '_')}
  echo "== $name"
  env ${lib:+HB_LIB_PATH=$lib} $envs timeout -k 10 300 python -u bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-parity-sample ${GIB:+--gib $GIB} > $OUT/$name.log 2>&1 || { echo "   FAILED"; tail -5 $OUT/$name.log; exit 1; }
  grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*' $OUT/$name.log | tr '\n' ' '; echo
done
if [ -n "$PMC" ]; then
  lib=""; [ "$PMCV" != base ] && lib=$PWD/exp_$PMCV.so
  i=0
  IFS=';' read -ra SETS <<< "$PMC"
  for set in "${SETS[@]}"; do
    i=$((i+1)); echo "== pmc $i: $set"
    HB_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc $set -d $OUT/pmc_$i -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity-sample --gib ${PMCGIB:-16} > $OUT/pmc_$i.log 2>&1 || { echo "   pmc FAILED"; exit 1; }
  done
fi
echo done
