#!/bin/bash
# Build the library from HEAD's sources into ctclip_mi355x/libctclip_hip_old.so (A/B timing with
# CTCLIP_HIP_LIB), leaving the working tree's build in libctclip_hip.so.   usage: tools/ab_build.sh [git-ref]
set -e
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
git archive "${1:-HEAD}" ctpa-clip_amd/csrc include | tar -x -C "$tmp"
make -s -C "$tmp/ctpa-clip_amd/csrc" -j8 OUT="$PWD/ctpa-clip_amd/ctclip_mi355x/libctclip_hip_old.so" >/dev/null
rm -rf "$tmp"
