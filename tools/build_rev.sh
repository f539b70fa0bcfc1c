#!/bin/bash
# Build libdeequ_amd.so from a git revision (or the working tree with rev "WT") into
# gpurun_ab/lib_<name>.so, for same-box A/B runs (DEEQU_AMD_LIB=...).  Usage: build_rev.sh <name> <rev>
set -eu
cd "$(dirname "$0")/.."
name=$1; rev=$2
tmp=$(mktemp -d)
if [ "$rev" = WT ]; then
  mkdir -p "$tmp/deequ_amd" "$tmp/include"
  cp -r deequ_amd/csrc "$tmp/deequ_amd/"; cp include/*.h "$tmp/include/"
else
  git archive "$rev" deequ_amd/csrc include | tar -x -C "$tmp"
fi
rm -rf "$tmp/deequ_amd/csrc/build"
make -s -C "$tmp/deequ_amd/csrc" -j8 >/dev/null
mkdir -p gpurun_ab
cp "$tmp/deequ_amd/libdeequ_amd.so" "gpurun_ab/lib_$name.so"
rm -rf "$tmp"
echo "gpurun_ab/lib_$name.so"
