#!/usr/bin/env bash
# round-4 GPU job 13: the headline at qk-norm gains 1 / 2 / 3 / 4 (bench.py --qk-gain)
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 1 | cut -c1-200
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
for g in 1 2 3 4; do
  run gain$g 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none --qk-gain $g
done
