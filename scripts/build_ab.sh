#!/bin/bash
# Build the product library of another git revision for a same-box A/B (scripts/gpu_run.sh
# ab:<lib>:...): sources from `git archive <rev>`, objects in /tmp, the library at
# model-predictive-control-for-bipedal-locomotion_amd/mpc_bipedal/ab/libzmpc_<tag>.so.
# Usage: bash scripts/build_ab.sh <rev> <tag> [extra make args]
set -eu
REV=$1
TAG=$2
shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=model-predictive-control-for-bipedal-locomotion_amd
SRC=/tmp/zmpc_ab_$TAG
rm -rf "$SRC"
mkdir -p "$SRC" "$ROOT/$PKG/mpc_bipedal/ab"
git -C "$ROOT" archive "$REV" "$PKG/csrc" include | tar -x -C "$SRC"
make -s -C "$SRC/$PKG/csrc" -j8 OUT="$ROOT/$PKG/mpc_bipedal/ab/libzmpc_$TAG.so" \
  OBJDIR="$SRC/build" "$@"
echo "$PKG/mpc_bipedal/ab/libzmpc_$TAG.so"
