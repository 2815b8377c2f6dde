#!/bin/bash
# Round 4: socket power and gfx clock (amd-smi, ~0.5 s samples) during 300
# steps of bench c3 with the dense MFMA MAC (in-tree build) and with the
# Toeplitz MAC (exp_toeplitz.so, HB_MFMA_TOEPLITZ), alternating, on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4power}
mkdir -p $OUT
sample() {   # $1 = tag, runs until the file $OUT/$1.stop exists or 120 s
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
  echo "$tag rc=$rc"; tail -n 1 $OUT/$tag.log | cut -c1-200
  return $rc
}
for r in 1 2; do
  unset HB_LIB_PATH
  run dense_$r python -u bench.py --steps 300 --warmup 2 --no-cpu-baseline --no-parity-sample || exit 1
  HB_LIB_PATH=./exp_toeplitz.so run toeplitz_$r python -u bench.py --steps 300 --warmup 2 --no-cpu-baseline --no-parity-sample || exit 1
done
echo done
