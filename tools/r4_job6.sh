#!/usr/bin/env bash
# round-4 GPU job 6: attention-backward software pipeline (SR_BWD_SCHED) tests + training A/B
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  tail -n 4 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
run tbwd6 300 python -u -m pytest tests/test_attn_bwd_gpu.py -x -q -m gpu --timeout 250 --timeout-method thread
run kt_s0 400 env SR_BWD_SCHED=0 python tools/kbench.py train
run kt_s1 400 env SR_BWD_SCHED=1 python tools/kbench.py train
run kt_s0b 400 env SR_BWD_SCHED=0 python tools/kbench.py train
run kt_s1b 400 env SR_BWD_SCHED=1 python tools/kbench.py train
