# Interleaved kbench GEMM rounds under environment settings (ENVS: VAR=VALUE list, "-" = defaults).
#   ENVS="- SR_GEMM_GROUP_M=8" KB="gemm" bash tools/ab_gemm_env.sh
set -o pipefail
for i in 1 2; do
  for e in ${ENVS:?set ENVS}; do
    echo "== $e"
    if [ "$e" = "-" ]; then set --; else set -- "$e"; fi
    env "$@" timeout -k 10 200 python tools/kbench.py ${KB:-gemm} 2>/dev/null | grep -v amdgpu || exit 1
  done
done
