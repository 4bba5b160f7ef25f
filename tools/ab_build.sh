#!/bin/bash
# Build an A/B variant of libmhppo.so into build_ab/<name>/ with extra compiler flags.
# usage: bash tools/ab_build.sh <name> "<flags>"
set -e
make -s -C "$(dirname "$0")/../mh-ppo_amd/csrc" -j8 BUILD="$PWD/build_ab/$1/obj" OUT="$PWD/build_ab/$1/libmhppo.so" EXTRA="$2" 2>&1 | grep -E "error" || true
ls -la build_ab/$1/libmhppo.so
