# A/B of the tuning variant library $VLIB against the shipped one on the whole bench step
# (interleaved runs on one box).
set -o pipefail
mkdir -p gpurun_out
VLIB=${VLIB:?set VLIB}
for i in 1 2; do
  echo "== shipped"; timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*\|"gemm_all_tflops": [0-9.]*' | tr '\n' ' '; echo
  echo "== $VLIB"; SFM_AMD_LIB=$VLIB timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*\|"gemm_all_tflops": [0-9.]*' | tr '\n' ' '; echo
done
