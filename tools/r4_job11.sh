#!/usr/bin/env bash
# round-4 GPU job 11: proj residual folded into LN2 (SR_FUSED_RESID_LN=1, optionally with the
# non-temporal residual-LN variant) vs the fused GEMM epilogue, with the tail split on
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 1 | cut -c1-300
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
B="python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none"
for i in 1 2; do
  run f0_$i 300 env SR_FUSED_RESID_LN=0 $B
  run f1_$i 300 env SR_FUSED_RESID_LN=1 $B
  run f1nt_$i 300 env SR_FUSED_RESID_LN=1 SR_RLN_WIDE=4 $B
done
