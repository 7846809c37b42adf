# Attention A/B job: attention tests under the default config and each SR_ATTN_CFG in $CFGS,
# then interleaved kbench attn rounds: $VLIBS (variant libraries), shipped, shipped x each cfg.
#   CFGS="3" VLIBS="self-supervise-sfm_amd/variants/lib_OLDATTN.so" bash tools/ab_attn_cfg.sh
set -o pipefail
mkdir -p gpurun_out
for c in - $CFGS; do
  e=""; [ "$c" = "-" ] || e="SR_ATTN_CFG=$c"
  env $e timeout -k 10 600 python -u -m pytest tests/test_baseline_shapes_gpu.py tests/test_kernels_gpu.py -x -q -m gpu \
    -k "attention or merge" --timeout 300 --timeout-method thread > gpurun_out/attn_tests_$c.log 2>&1 \
    || { tail -30 gpurun_out/attn_tests_$c.log; exit 1; }
  echo "tests cfg $c: $(tail -1 gpurun_out/attn_tests_$c.log)"
done
for i in 1 2; do
  for v in $VLIBS; do
    echo "== $v"; SFM_AMD_LIB=$v SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py ${KB:-attn} 2>/dev/null | grep -v amdgpu || exit 1
  done
  for c in - $CFGS; do
    e=""; [ "$c" = "-" ] || e="SR_ATTN_CFG=$c"
    echo "== cfg $c"; env $e SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py ${KB:-attn} 2>/dev/null | grep -v amdgpu || exit 1
  done
done
