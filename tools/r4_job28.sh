#!/usr/bin/env bash
# round-4 GPU job 28: the persistent 256x256 GEMM (SR_GEMM_PERSIST): parity, kbench A/B, bench A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "gemm|passed|failed|value" "gpurun_out/$name.log" | grep -v kernel_breakdown | cut -c1-300 | tail -n 14
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 30 "gpurun_out/$name.log"; exit $rc; fi
}
run j28_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -k "gemm_persistent or gemm_tail" tests/test_kernels_gpu.py
run j28_k0 200 python tools/kbench.py gemm gemm_k
SR_GEMM_PERSIST=1 run j28_k1 200 python tools/kbench.py gemm gemm_k
run j28_b0 300 python bench.py --steps 6 --warmup 2 --extras none --no-cpu-baseline
SR_GEMM_PERSIST=1 run j28_b1 300 python bench.py --steps 6 --warmup 2 --extras none --no-cpu-baseline
run j28_b0b 300 python bench.py --steps 6 --warmup 2 --extras none --no-cpu-baseline
SR_GEMM_PERSIST=1 run j28_b1b 300 python bench.py --steps 6 --warmup 2 --extras none --no-cpu-baseline
