#!/usr/bin/env bash
# round-5 GPU job 7: the 256x256 GEMM's ping-pong k-loop (SR_GEMM_PP): bit-identity tests, kbench A/B.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|gemm_pp" "gpurun_out/$name.log" | cut -c1-200 | tail -n 24
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j7_tests 300 python -u -m pytest tests/test_kernels_gpu.py -q -s -m gpu -k "ping_pong" --timeout 120 --timeout-method thread
run j7_kpp 300 python tools/kbench.py gemm_pp
