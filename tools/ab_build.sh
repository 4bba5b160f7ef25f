#!/bin/bash
# Build an alternative libmhppo.so for A/B kernel experiments:
#   tools/ab_build.sh <name> "<extra hipcc flags>"  ->  build_ab/<name>/libmhppo.so
# then run with MHPPO_LIB=build_ab/<name>/libmhppo.so (mhppo/_lib.py).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
make -s -C "$ROOT/mh-ppo_amd/csrc" OUT="$ROOT/build_ab/$NAME/libmhppo.so" BUILD="$ROOT/build_ab/$NAME/obj" EXTRA="$*"
