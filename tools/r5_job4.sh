#!/usr/bin/env bash
# round-5 GPU job 4: the few-row fp32 GEMM (sr_gemm_skinny_f32, camera trunk) and the residual GEMMs'
# x prefetch (SR_GEMM_XPF): kernel tests, kbench gemm_cam / gemm_qkv (RoPE tables in LDS or not) /
# gemm_xpf, parity + camera-head backward, the step A/B for each, the per-rank rehearsal at G = 8.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"|skinny|step_ms|xpf|gemm_qkv" "gpurun_out/$name.log" | cut -c1-220 | tail -n 14
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j4_tests 600 python -u -m pytest tests/test_kernels_gpu.py -q -s -m gpu -k "skinny or splitk or bias_gelu or x_prefetch or gemm_group or tail_split or qkv" --timeout 300 --timeout-method thread
run j4_kcam 300 python tools/kbench.py gemm_cam
run j4_kqkv 300 python tools/kbench.py gemm_qkv
run j4_xpf 300 python tools/kbench.py gemm_xpf
run j4_parity 600 python -u -m pytest tests/test_parity_gpu.py tests/test_train_graph_gpu.py -q -s -m gpu --timeout 500 --timeout-method thread
for i in 1 2; do
  SR_GEMM_SKINNY=0 run j4_bench_s0_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  run j4_bench_s1_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  SR_GEMM_XPF=-1 run j4_bench_xa_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
SR_GROUP_TAILS=0 SR_GEMM_SKINNY=0 run j4_rs_base 300 python tools/rank_sim.py --worlds 8 --steps 5 --warmup 2
run j4_rs_new 300 python tools/rank_sim.py --worlds 8 --steps 5 --warmup 2
