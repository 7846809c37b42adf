#!/usr/bin/env bash
# round-5 GPU job 27: the layer's reloc + global backward with grouped dgrad GEMMs
# (SR_TRAIN_PAIR_DGRAD=1): grouped-epilogue tests, the training tests, training A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|ms/step|dgrad" "gpurun_out/$name.log" | cut -c1-160 | tail -n 14
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j27_group 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm_group" --timeout 120 --timeout-method thread
run j27_train_tests 700 python -u -m pytest tests/test_train_step_gpu.py tests/test_c4_golden_gpu.py -x -q -m gpu --timeout 600 --timeout-method thread
run j27_train1 400 python tools/kbench.py train
SR_TRAIN_PAIR_DGRAD=0 run j27_train0 400 python tools/kbench.py train
