#!/bin/bash
# Build libdeequ_amd.so with extra compile flags into gpurun_ab/lib_<name>.so for same-box A/B
# runs (tools/ab.sh, DEEQU_AMD_LIB).  Usage: tools/build_variant.sh <name> "<-DFLAG=1 ...>" ["<sed script>"]
# The optional sed script edits the COPY of dq_freq.hip only (timing probes such as "skip this
# step": results wrong, never shipped -- the tree's sources are untouched).
set -eu
cd "$(dirname "$0")/.."
name=$1; flags=${2:-}
tmp=$(mktemp -d)
mkdir -p "$tmp/deequ_amd" "$tmp/include"
cp -r deequ_amd/csrc "$tmp/deequ_amd/"
cp include/*.h "$tmp/include/"
rm -rf "$tmp/deequ_amd/csrc/build"
if [ -n "${3:-}" ]; then sed -i "$3" "$tmp/deequ_amd/csrc/dq_freq.hip"; fi
make -s -C "$tmp/deequ_amd/csrc" -j8 CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function $flags" >/dev/null
mkdir -p gpurun_ab
cp "$tmp/deequ_amd/libdeequ_amd.so" "gpurun_ab/lib_$name.so"
rm -rf "$tmp"
echo "gpurun_ab/lib_$name.so"
