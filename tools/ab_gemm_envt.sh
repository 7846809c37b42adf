# GEMM env A/B job: GEMM (+ parity) tests under each environment setting in $ENVS ("-" = defaults),
# then interleaved kbench gemm rounds.   ENVS="- SR_GEMM_PERSIST=1" bash tools/ab_gemm_envt.sh
set -o pipefail
mkdir -p gpurun_out
for e in ${ENVS:?set ENVS}; do
  [ "$e" = "-" ] && continue
  env $e timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_parity_gpu.py -x -q -m gpu \
    -k "${TK:-gemm or c2 or 518}" --timeout 300 --timeout-method thread > gpurun_out/gemm_envt_tests.log 2>&1 \
    || { tail -30 gpurun_out/gemm_envt_tests.log; exit 1; }
  echo "tests $e: $(tail -1 gpurun_out/gemm_envt_tests.log)"
done
for i in 1 2; do
  for e in $ENVS; do
    echo "== $e"
    if [ "$e" = "-" ]; then set --; else set -- "$e"; fi
    env "$@" timeout -k 10 200 python tools/kbench.py ${KB:-gemm} 2>/dev/null | grep -v amdgpu || exit 1
  done
done
