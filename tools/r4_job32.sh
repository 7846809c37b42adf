#!/usr/bin/env bash
# round-4 GPU job 32: one weight-refresh launch per block (casts + transposed dgrad packs); colsum
# chunks: training-kernel parity, the C4 golden, and the training step
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|train:|Error" "gpurun_out/$name.log" | cut -c1-300 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
}
run j32_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -k "layernorm or not test_kernels_gpu" tests/test_kernels_gpu.py tests/test_train_kernels_gpu.py tests/test_train_graph_gpu.py tests/test_train_step_gpu.py tests/test_train_block_gpu.py tests/test_c4_golden_gpu.py
run j32_train1 300 python tools/kbench.py train
run j32_train2 300 python tools/kbench.py train
