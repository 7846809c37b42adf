#!/usr/bin/env bash
# round-5 GPU job 31: the reloc + global blocks' weight grads paired in one launch (SR_TRAIN_PAIR_WGRAD):
# wgrad pair tests, C4 golden / train-step tests, training A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|ms/step|wgrad" "gpurun_out/$name.log" | cut -c1-160 | tail -n 12
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j31_tests 300 python -u -m pytest tests/test_train_kernels_gpu.py tests/test_c4_golden_gpu.py tests/test_train_step_gpu.py -x -q -m gpu -k "wgrad or c4 or train" --timeout 200 --timeout-method thread
run j31_train_w1a 400 python tools/kbench.py train
SR_TRAIN_PAIR_WGRAD=0 run j31_train_w0 400 python tools/kbench.py train
run j31_train_w1b 400 python tools/kbench.py train
