#!/usr/bin/env bash
# round-5 GPU job 24: key-split chunk alignment modes 2 / 3 (p whole-tile chunks + a short
# remainder) against equal chunks, rank-0 rehearsal G = 4, 8, interleaved, 2 runs each
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  python3 -c "
import json,sys
for l in open('gpurun_out/$name.log'):
    if l.startswith('{\"world\"'):
        d=json.loads(l); print(d['world'], d['step_ms'], d['kernel_ms_per_step'].get('attn_global'), d['kernels'].get('attn_global'))
"
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
for i in 1 2; do
  run j24_rs_a0_$i 300 python tools/rank_sim.py --worlds 4,8 --steps 5 --warmup 2
  SR_SHARD_ALIGN=2 run j24_rs_a2_$i 300 python tools/rank_sim.py --worlds 4,8 --steps 5 --warmup 2
  SR_SHARD_ALIGN=3 run j24_rs_a3_$i 300 python tools/rank_sim.py --worlds 4,8 --steps 5 --warmup 2
done
