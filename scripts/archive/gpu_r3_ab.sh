#!/bin/bash
# Round-3 session: VALU issue-class microbench, then A/B of the byte-1
# address variants against the in-tree build (scripts/gpu_ab.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3ab}
mkdir -p $OUT
if [ -z "$NOUBENCH" ]; then
  echo "== ubench_valu"
  timeout -k 10 120 ./scripts/ubench_valu > $OUT/valu_rates.log 2>&1 || { echo "ubench failed"; exit 1; }
  cat $OUT/valu_rates.log
fi
TAG=${TAG:-r3ab} bash scripts/gpu_ab.sh
