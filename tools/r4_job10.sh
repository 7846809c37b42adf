#!/usr/bin/env bash
# round-4 GPU job 10: backward tests after removing the schedule variants; one full N=32 oracle
# forward on the box's host cores (tools/cpu_full.py)
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
run tbwd10 300 python -u -m pytest tests/test_attn_bwd_gpu.py tests/test_train_block_gpu.py -x -q -m gpu --timeout 250 --timeout-method thread
run cpu_full 1000 python -u tools/cpu_full.py
