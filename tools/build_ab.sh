#!/usr/bin/env bash
# Build libsfm_amd.so from a git revision's csrc + include (default HEAD) into ab/libsfm_<name>.so,
# for same-process / same-box A/B runs against the working tree's build (load it with
# SFM_AMD_LIB=ab/libsfm_<name>.so).  ab/ is git-ignored but travels to the GPU box.
#   tools/build_ab.sh base [REV]
set -eu
name=$1; rev=${2:-HEAD}
repo=$(cd "$(dirname "$0")/.." && pwd)
work=$(mktemp -d /tmp/sfm_ab_XXXX)
git -C "$repo" archive "$rev" self-supervise-sfm_amd/csrc include | tar -x -C "$work"
mkdir -p "$repo/ab"
make -s -C "$work/self-supervise-sfm_amd/csrc" -j8 OUT="$repo/ab/libsfm_$name.so" BUILD="$work/build" \
  > "$work/make.log" 2>&1 || { tail -30 "$work/make.log"; exit 1; }
rm -rf "$work"
echo "built ab/libsfm_$name.so from $rev"
