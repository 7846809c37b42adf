#!/usr/bin/env bash
# round-5 GPU job 29: the layer's reloc + global training forward grouped (SR_TRAIN_PAIR_FWD):
# grouped-GEMM aux tests, C4 golden / train-step tests, training A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|ms/step|gemm_" "gpurun_out/$name.log" | cut -c1-160 | tail -n 12
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j29_tests 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_c4_golden_gpu.py tests/test_train_step_gpu.py -x -q -m gpu -k "gemm_group or c4 or train" --timeout 200 --timeout-method thread
run j29_train_f1a 400 python tools/kbench.py train
SR_TRAIN_PAIR_FWD=0 run j29_train_f0 400 python tools/kbench.py train
run j29_train_f1b 400 python tools/kbench.py train
