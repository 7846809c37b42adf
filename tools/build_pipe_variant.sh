#!/usr/bin/env bash
# Build an A/B variant of libsfm_amd.so whose hand-scheduled attention sweep is generated with the
# given generator knobs (tools/gen_attn_pipe.py environment), into variants/libsfm_<name>.so.
#   tools/build_pipe_variant.sh vb128 SR_PIPE_EXP_VB128=1
# Load it with SFM_AMD_LIB=variants/libsfm_<name>.so (tools/gpu_job.sh kattn_var).
set -eu
name=$1; shift
repo=$(cd "$(dirname "$0")/.." && pwd)
work=$(mktemp -d /tmp/sfm_var_XXXX)
mkdir -p "$work/pkg"
cp -r "$repo/self-supervise-sfm_amd/csrc" "$work/pkg/csrc"
mkdir -p "$work/include" "$repo/variants"
cp "$repo/include/sfm_amd.h" "$work/include/"
env "$@" SR_PIPE_OUT="$work/pkg/csrc/sr_attn_pipe.inc" python3 "$repo/tools/gen_attn_pipe.py"
make -s -C "$work/pkg/csrc" -j8 OUT="$repo/variants/libsfm_$name.so" BUILD="$work/build" \
  > "$work/make.log" 2>&1 || { tail -30 "$work/make.log"; exit 1; }
rm -rf "$work"
echo "built variants/libsfm_$name.so"
