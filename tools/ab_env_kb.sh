# Interleaved kbench rounds under environment settings, no tests (timing-only A/B).
#   ENVS="- SR_ATTN_KSPLIT=2" KB=attn bash tools/ab_env_kb.sh
set -o pipefail
for i in 1 2; do
  for e in ${ENVS:?set ENVS}; do
    echo "== $e"
    if [ "$e" = "-" ]; then set --; else set -- "$e"; fi
    env SR_KB_STATIC=1 "$@" timeout -k 10 200 python tools/kbench.py ${KB:-attn} 2>/dev/null | grep -v amdgpu || exit 1
  done
done
