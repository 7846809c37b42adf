#!/usr/bin/env bash
# round-5 GPU job 4: the few-row fp32 GEMM (sr_gemm_skinny_f32, camera trunk): kernel tests, kbench
# gemm_cam (old split-K sweep + the new kernel), camera-head parity, and the step with the new
# kernel on / off (SR_GEMM_SKINNY), interleaved; the per-rank rehearsal at G = 8 on / off.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"|skinny|step_ms|qtail|xpf" "gpurun_out/$name.log" | cut -c1-220 | tail -n 12
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j4_tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_baseline_shapes_gpu.py -q -s -m gpu -k "skinny or splitk or bias_gelu or q_tail or x_prefetch or gemm_group or tail_split" --timeout 300 --timeout-method thread
run j4_kcam 300 python tools/kbench.py gemm_cam
run j4_qtail 300 python tools/kbench.py attn_qtail
run j4_parity 900 python -u -m pytest tests/test_parity_gpu.py tests/test_layers_gpu.py tests/test_train_graph_gpu.py tests/test_c4_golden_gpu.py -q -s -m gpu --timeout 600 --timeout-method thread
for i in 1 2; do
  SR_GEMM_SKINNY=0 run j4_bench_s0_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  run j4_bench_s1_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
SR_GEMM_SKINNY=0 run j4_rs_s0 300 python tools/rank_sim.py --worlds 8 --steps 5 --warmup 2
run j4_rs_s1 300 python tools/rank_sim.py --worlds 8 --steps 5 --warmup 2
# the residual GEMMs' x prefetch (SR_GEMM_XPF): kbench, then the step (default 0 vs auto)
run j4_xpf 300 python tools/kbench.py gemm_xpf
for i in 1 2; do
  run j4_bench_x0_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  SR_GEMM_XPF=-1 run j4_bench_xa_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
