#!/usr/bin/env bash
# round-4 GPU job 1: the new attention tests, qk-gain kbench, LN kbench, deferred-residual A/B
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
run t1 600 python -u -m pytest tests/test_baseline_shapes_gpu.py tests/test_layers_gpu.py -x -v -m gpu --timeout 300 \
    --timeout-method thread -k "qk_gain or bit31 or pair or static_key or global_attention_production or reloc_attention_production or frame_attention_production or fully_masked"
run k1 300 python tools/kbench.py attn_gain attn_pair ln
run t2 600 python -u -m pytest tests/test_parity_gpu.py tests/test_kernels_gpu.py -x -v -m gpu --timeout 300 \
    --timeout-method thread -k "deferred or residual_layernorm or block_kats"
for i in 1 2; do
  run bench_d0_$i 300 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
  run bench_d1_$i 300 env SR_FUSED_RESID_LN=1 SR_DEFER_RESID=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
done
