#!/usr/bin/env bash
# round-5 GPU job 5: the frame-sharded path with the grouped global Q + K/V GEMM and the grouped
# global + reloc tails (sharded tests; per-rank rehearsal A/B against SR_GEMM_GROUP=0, which turns
# every grouped launch off), and the default step after dropping the few-row fp32 GEMM.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"|step_ms" "gpurun_out/$name.log" | cut -c1-160 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j5_tests 600 python -u -m pytest tests/test_kernels_gpu.py -q -s -m gpu -k "splitk or bias_gelu or gemm_group" --timeout 300 --timeout-method thread
run j5_dist 900 python -u -m pytest tests/test_dist_gpu.py -q -s -m gpu --timeout 600 --timeout-method thread
for i in 1 2; do
  SR_GEMM_GROUP=0 run j5_rs_g0_$i 300 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
  run j5_rs_g1_$i 300 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
done
run j5_bench_1 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
run j5_kcam 300 python tools/kbench.py gemm_cam
