#!/usr/bin/env bash
# round-4 GPU job 34: key and value boxes on key-scan launches (training forward); colsum
# chunks: training-kernel parity, the C4 golden, and the training step
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|train:|attn_global |Error|scan mode" "gpurun_out/$name.log" | cut -c1-300 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
}
run j34_tests 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -k "layernorm or scan_boxes or key_box or value_window or qk_gain or not (test_kernels_gpu or test_baseline_shapes_gpu)" tests/test_kernels_gpu.py tests/test_baseline_shapes_gpu.py tests/test_train_kernels_gpu.py tests/test_train_graph_gpu.py tests/test_train_step_gpu.py tests/test_train_block_gpu.py tests/test_c4_golden_gpu.py
run j34_train1 300 python tools/kbench.py train
run j34_train2 300 python tools/kbench.py train
SR_TRAIN_QK_GAIN=4 run j34_train_g4 300 python tools/kbench.py train
SR_ATTN_KEY_BOX=0 SR_TRAIN_QK_GAIN=4 run j34_train_g4_nobox 300 python tools/kbench.py train
