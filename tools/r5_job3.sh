#!/usr/bin/env bash
# round-5 GPU job 3: QKV epilogue (RoPE tables in LDS, row-swap permutes for the head LayerNorm):
# GEMM / QKV kernel tests and the C3 goldens on the new build, then kbench gemm_qkv A/B against the
# previous build (ab/libsfm_base.so), interleaved, and the step; the attention q-tail launch
# (SR_ATTN_QTAIL); the grouped global + reloc tails under frame sharding (SR_GROUP_TAILS).
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"|gemm_qkv|step_ms" "gpurun_out/$name.log" | cut -c1-200 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j3_tests 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py tests/test_layers_gpu.py -q -s -m gpu -k "gemm or qkv or full_c3 or small or block or attention_layer or Attention" --timeout 600 --timeout-method thread
run j3_shapes 600 python -u -m pytest tests/test_baseline_shapes_gpu.py -q -s -m gpu -k "q_tail or frame_attention or reloc_attention" --timeout 300 --timeout-method thread
run j3_qtail 200 python tools/kbench.py attn_qtail
run j3_dist 900 python -u -m pytest tests/test_dist_gpu.py -q -s -m gpu --timeout 600 --timeout-method thread
for i in 1 2; do
  SFM_AMD_LIB=ab/libsfm_base.so run j3_kq_base_$i 200 python tools/kbench.py gemm_qkv
  run j3_kq_new_$i 200 python tools/kbench.py gemm_qkv
done
for i in 1 2; do
  SFM_AMD_LIB=ab/libsfm_base.so run j3_bench_base_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  run j3_bench_new_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
# frame-sharded per-rank rehearsal: the global + reloc tails grouped (SR_GROUP_TAILS=1, default) or not
for i in 1 2; do
  SR_GROUP_TAILS=0 run j3_rs_g0_$i 400 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
  run j3_rs_g1_$i 400 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
done
