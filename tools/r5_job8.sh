#!/usr/bin/env bash
# round-5 GPU job 8: the ping-pong k-loop (SR_GEMM_PP) in the whole step, interleaved, plus the group
# kernel's bit-identity.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"" "gpurun_out/$name.log" | cut -c1-160 | tail -n 4
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
SR_GEMM_PP=1 run j8_tests 300 python -u -m pytest tests/test_kernels_gpu.py -q -s -m gpu -k "gemm_group or ping_pong or tail_split" --timeout 120 --timeout-method thread
for i in 1 2 3; do
  run j8_bench_pp0_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  SR_GEMM_PP=1 run j8_bench_pp1_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
