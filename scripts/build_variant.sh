#!/bin/bash
# Build an A/B variant of libhbswizzle.so as exp_<name>.so at the repo root
# (git-ignored; loaded by bench.py / gpu_exp.sh through HB_LIB_PATH).
#   scripts/build_variant.sh <name> <extra hipcc flags...>
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$ROOT/heartbeat_amd/csrc" -j${JOBS:-4} NL64=${NL64:-0} BUILD=build_$name OUT=../../exp_$name.so \
  FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-pass-failed -DHB_EXPERIMENT_BUILD $*"
echo "built exp_$name.so"
