#!/usr/bin/env bash
# round-5 GPU job 12: grouped tails at every G (SR_GROUP_TAILS=2) against the default (1: blocks of
# <= 16,384 rows), the same worlds in both arms, interleaved.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|step_ms" "gpurun_out/$name.log" | cut -c1-130 | tail -n 5
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
for i in 1 2; do
  run j12_rs_g1_$i 400 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
  SR_GROUP_TAILS=2 run j12_rs_g2_$i 400 python tools/rank_sim.py --worlds 2,4,8 --steps 5 --warmup 2
done
