set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_baseline_shapes_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -k "attention or merge" --timeout 300 --timeout-method thread > gpurun_out/kb_tests.log 2>&1 || { tail -30 gpurun_out/kb_tests.log; exit 1; }
tail -1 gpurun_out/kb_tests.log
for i in 1 2; do
echo "== scan"; timeout -k 10 200 python tools/kbench.py attn || exit 1
echo "== static"; SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py attn || exit 1
done
