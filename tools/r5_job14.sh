#!/usr/bin/env bash
# round-5 GPU job 14: the attention backward's dK/dV sweep with two key blocks per wave
# (SR_ATTN_BWD_KB=2): bit-identity and autograd tests, kbench A/B, the training step A/B.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|attn_bwd|ms/step" "gpurun_out/$name.log" | cut -c1-160 | tail -n 10
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j14_tests 300 python -u -m pytest tests/test_attn_bwd_gpu.py -q -s -m gpu --timeout 200 --timeout-method thread
run j14_kbwd 300 python tools/kbench.py attn_bwd
run j14_train1 400 python tools/kbench.py train
SR_ATTN_BWD_KB=2 run j14_train2 400 python tools/kbench.py train
