#!/usr/bin/env bash
# Time tools/kbench.py <what> against the stock library and each tuning build in
# self-supervise-sfm_amd/variants/ (make -C self-supervise-sfm_amd/csrc variants).
# Stops at the first crash / timeout.
#   tools/ablate.sh attn [NOEXP NOPV ...]
set -u
what=$1; shift
mkdir -p gpurun_out
out=gpurun_out/ablate_$what.log
: > "$out"
libs=("")
if [ $# -gt 0 ]; then for v in "$@"; do libs+=("self-supervise-sfm_amd/variants/lib_$v.so"); done
else for f in self-supervise-sfm_amd/variants/lib_*.so; do libs+=("$f"); done; fi
for lib in "${libs[@]}"; do
  echo "=== ${lib:-stock}" | tee -a "$out"
  SFM_AMD_LIB="$lib" timeout -k 10 240 python tools/kbench.py "$what" 2>&1 | grep -v amdgpu.ids | tee -a "$out"
  rc=${PIPESTATUS[0]}
  if [ "$rc" -ne 0 ]; then echo "=== rc=$rc: stopping" | tee -a "$out"; exit "$rc"; fi
done
