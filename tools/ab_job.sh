# A/B job: the tuning variant library $VLIB against the shipped one (attention tests + kbench attn)
set -o pipefail
mkdir -p gpurun_out
VLIB=${VLIB:-self-supervise-sfm_amd/variants/lib_MSUM.so}
[ -n "$SKIPTEST" ] || SFM_AMD_LIB=$VLIB timeout -k 10 600 python -u -m pytest tests/test_baseline_shapes_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -k "attention or merge" --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
[ -n "$SKIPTEST" ] || tail -1 gpurun_out/ab_tests.log
for i in 1 2; do
echo "== shipped"; SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py attn || exit 1
echo "== $VLIB"; SFM_AMD_LIB=$VLIB SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py attn || exit 1
done
