#!/bin/bash
# Socket power and clocks while the encode (bench c3, many steps) and the
# T-table / bitsliced / mixed AES microbench configurations run; amd-smi (or
# rocm-smi) sampled every ~0.5 s.  Every step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-power}
mkdir -p $OUT
timeout -k 5 20 amd-smi metric -g 0 --json > $OUT/amdsmi_idle.json 2>&1; echo "amd-smi rc=$?"
timeout -k 5 20 rocm-smi --showpower --showclocks --json > $OUT/rocmsmi_idle.json 2>&1; echo "rocm-smi rc=$?"
sample() {   # $1 = tag, runs until the file $OUT/$1.stop exists or 120 s
  local t0=$(date +%s.%N)
  for i in $(seq 1 240); do
    [ -e $OUT/$1.stop ] && break
    echo "== $(date +%s.%N)" >> $OUT/$1.power
    timeout -k 2 5 amd-smi metric -g 0 -p -c --json >> $OUT/$1.power 2>&1
    sleep 0.3
  done
}
run() {   # $1 = tag, rest = command
  local tag=$1; shift
  sample $tag &
  local sp=$!
  timeout -k 10 150 "$@" > $OUT/$tag.log 2>&1; local rc=$?
  touch $OUT/$tag.stop; wait $sp
  echo "$tag rc=$rc"; tail -n 2 $OUT/$tag.log | cut -c1-300
  return $rc
}
run encode python -u bench.py --steps 300 --warmup 2 --no-cpu-baseline --no-parity-sample || exit 1
HB_BS_SECONDS=8 HB_BS_ONLY="T-table 16" run bs_ttable ./scripts/bitslice/ubench_bs || exit 1
HB_BS_SECONDS=8 HB_BS_ONLY="bitsliced 16" run bs_bitsliced ./scripts/bitslice/ubench_bs || exit 1
HB_BS_SECONDS=8 HB_BS_ONLY="mixed 8 T" run bs_mixed ./scripts/bitslice/ubench_bs || exit 1
echo done
