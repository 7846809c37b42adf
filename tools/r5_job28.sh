#!/usr/bin/env bash
# round-5 GPU job 28: the 3-stage 48-row wgrad (SR_WGRAD_STAGES=3): wgrad tests, training A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|ms/step|wgrad" "gpurun_out/$name.log" | cut -c1-160 | tail -n 10
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j28_tests 200 python -u -m pytest tests/test_train_kernels_gpu.py -x -q -m gpu -k "wgrad" --timeout 120 --timeout-method thread
run j28_train2 400 python tools/kbench.py train
SR_WGRAD_STAGES=3 run j28_train3 400 python tools/kbench.py train
