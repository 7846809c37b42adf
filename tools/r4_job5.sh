#!/usr/bin/env bash
# round-4 GPU job 5: attention-backward rework (scalar staging, -delta seeds, packed dS) tests +
# training kbench + C4 golden; residual-LN variants; GEMM tail split tests + A/B
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  tail -n 4 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
run tbwd 400 python -u -m pytest tests/test_attn_bwd_gpu.py tests/test_train_block_gpu.py tests/test_train_graph_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread
run ktrain 400 python tools/kbench.py train
run tc4 400 python -u -m pytest tests/test_c4_golden_gpu.py -x -q -s -m gpu --timeout 350 --timeout-method thread
run tln 200 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "residual_layernorm or gemm_tail or gemm_group or gemm256"
run kln 200 python tools/kbench.py ln attn_frame_cfg
run b_t0a 300 env SR_GEMM_TAIL=0 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run b_t1a 300 env SR_GEMM_TAIL=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run b_t0b 300 env SR_GEMM_TAIL=0 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run b_t1b 300 env SR_GEMM_TAIL=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run rs_t1 200 env SR_GEMM_TAIL=1 python tools/rank_sim.py --views 32 --worlds 2,4,8 --steps 4
