# Interleaved bench runs under environment settings on one box: ENVS is a space-separated list of
# VAR=VALUE settings ("-" = the shipped defaults), ARGS extra bench.py arguments.
#   ENVS="- SR_ATTN_KSPLIT=0" ARGS="--views 8" bash tools/ab_env.sh
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for e in ${ENVS:?set ENVS}; do
    echo "== $e"
    if [ "$e" = "-" ]; then set --; else set -- "$e"; fi
    env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${ARGS:-} 2>/dev/null \
      > gpurun_out/ab_env_last.log || exit 1
    python - <<'PY'
import json
for line in open("gpurun_out/ab_env_last.log"):
    if line.startswith('{"kernel_breakdown'):
        kb = json.loads(line)["kernel_breakdown"]
        print("  ", {k: v["avg_ms"] for k, v in kb.items() if k.startswith("attn")})
    elif line.startswith('{"metric'):
        print("   value", round(json.loads(line)["value"], 2))
PY
  done
done
