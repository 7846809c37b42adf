#!/usr/bin/env bash
# round-5 GPU job 10: the frame-sharded reloc attention on a second stream beside the global attention
# (SR_SHARD_CONCURRENT=1): per-rank rehearsal A/B, then the sharded GPU tests with it.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|step_ms" "gpurun_out/$name.log" | cut -c1-130 | tail -n 4
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
for i in 1 2; do
  run j10_rs_c0_$i 300 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
  SR_SHARD_CONCURRENT=1 run j10_rs_c1_$i 300 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
done
SR_SHARD_CONCURRENT=1 run j10_dist 900 python -u -m pytest tests/test_dist_gpu.py -q -s -m gpu --timeout 600 --timeout-method thread
