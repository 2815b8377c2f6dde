#!/bin/bash
# Round 4: rehearsal of the N-rank bench path on the one-GPU box (every rank on
# device 0, HB_BENCH_SAME_DEVICE=1): configs[3]'s plan (the --gpus N > 1
# default, c4) with a small per-rank share, self-spawned (4 ranks) and under
# torch.distributed.run (2 ranks).  The N = 8 node run is the driver's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r4reh}
mkdir -p $OUT
step() { local name=$1 limit=$2; shift 2; echo "== $name"; timeout -k 10 $limit "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "   rc=$rc"; tail -1 $OUT/$name.log | cut -c1-400; return $rc; }
export HB_BENCH_SAME_DEVICE=1
step reh_spawn4 300 python -u bench.py --gpus 4 --gib 2 --steps 2 --no-cpu-baseline || exit 1
step reh_torchrun2 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --gib 2 --steps 2 --no-cpu-baseline || exit 1
echo done
