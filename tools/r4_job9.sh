#!/usr/bin/env bash
# round-4 GPU job 9: hand-ordered dK/dV tile (SR_BWD_SCHED=1) tests + A/B
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
T="--timeout 300 --timeout-method thread"
run tbwd9 300 python -u -m pytest tests/test_attn_bwd_gpu.py tests/test_train_block_gpu.py -x -q -m gpu $T
run kb_s0 120 env SR_BWD_SCHED=0 python tools/kbench.py attn_bwd
run kb_s1 120 env SR_BWD_SCHED=1 python tools/kbench.py attn_bwd
run kb_s0b 120 env SR_BWD_SCHED=0 python tools/kbench.py attn_bwd
run kb_s1b 120 env SR_BWD_SCHED=1 python tools/kbench.py attn_bwd
export SR_BWD_SCHED=1
run pmc_s1a 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_s1a -o run --output-format csv -- python3 tools/kbench.py attn_bwd
