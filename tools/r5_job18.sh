#!/usr/bin/env bash
# round-5 GPU job 18: the hand-scheduled dQ sweep (SR_ATTN_BWD_DQ_PIPE=1): bit-identity tests
# first (short limit), then the rest of the backward tests, the kbench A/B and the training step.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|attn_bwd|ms/step" "gpurun_out/$name.log" | cut -c1-160 | tail -n 12
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j18_pipe 150 python -u -m pytest tests/test_attn_bwd_gpu.py -x -q -s -m gpu -k "pipe" --timeout 60 --timeout-method thread
run j18_tests 300 python -u -m pytest tests/test_attn_bwd_gpu.py -q -s -m gpu --timeout 200 --timeout-method thread
run j18_kbwd 300 python tools/kbench.py attn_bwd
run j18_train0 400 python tools/kbench.py train
SR_ATTN_BWD_DQ_PIPE=1 run j18_train1 400 python tools/kbench.py train
