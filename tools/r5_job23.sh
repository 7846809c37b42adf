#!/usr/bin/env bash
# round-5 GPU job 23: tile-aligned key chunks for the frame-sharded global attention
# (SR_SHARD_ALIGN=1): sharded GPU tests with it, then the rank-0 rehearsal A/B (G = 2, 4, 8),
# interleaved, 2 runs each
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|step_ms" "gpurun_out/$name.log" | cut -c1-220 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
SR_SHARD_ALIGN=1 run j23_dist 500 python -u -m pytest tests/test_dist_gpu.py -q -m gpu --timeout 400 --timeout-method thread
for i in 1 2; do
  run j23_rs_a0_$i 300 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
  SR_SHARD_ALIGN=1 run j23_rs_a1_$i 300 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
done
