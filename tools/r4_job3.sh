#!/usr/bin/env bash
# round-4 GPU job 3: residual-LN variants, frame cfg, backward + training-graph tests, training
# kbench, per-rank rehearsal A/B (reloc split threshold, asm ragged key-split passes), gain kbench
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
run ttrain 300 python -u -m pytest tests/test_train_graph_gpu.py -x -v -s -m gpu --timeout 250 --timeout-method thread
run tbwd 600 python -u -m pytest tests/test_attn_bwd_gpu.py tests/test_train_block_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread
run rs_base 200 python tools/rank_sim.py --views 32 --worlds 2,4,8 --steps 4
run rs_split 200 env SR_RELOC_SPLIT_MIN_WG=0 python tools/rank_sim.py --views 32 --worlds 2,4,8 --steps 4
run rs_tail 200 env SR_RELOC_SPLIT_MIN_WG=0 SR_SHARD_TAIL=1 python tools/rank_sim.py --views 32 --worlds 2,4,8 --steps 4
run ktrain 600 python tools/kbench.py train
run tln 200 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k residual_layernorm
run kln 200 python tools/kbench.py ln attn_frame_cfg
run k2 300 python tools/kbench.py attn_gain
run bench 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
