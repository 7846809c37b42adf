#!/usr/bin/env bash
# round-5 GPU job 35: the float4 Adam update:
# training kernel / C4 / train-step tests, two training runs, a kernel-stats profile of the step
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|train:" "gpurun_out/$name.log" | cut -c1-160 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j35_tests 500 python -u -m pytest tests/test_train_kernels_gpu.py tests/test_train_block_gpu.py tests/test_c4_golden_gpu.py tests/test_train_step_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread
run j35_train_a 400 python tools/kbench.py train
run j35_train_b 400 python tools/kbench.py train
SR_TRAIN_STEPS=4 run j35_prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/j35_prof -o run --output-format csv -- python3 tools/kbench.py train
