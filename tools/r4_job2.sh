#!/usr/bin/env bash
# round-4 GPU job 2: frame-sharded C3 / N=64 tests, per-rank rehearsal, training kbench
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  tail -n 4 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
run dist 700 python -u -m pytest tests/test_dist_gpu.py -x -v -s -m gpu --timeout 600 --timeout-method thread -k "c3 or n64"
run ranksim 250 python tools/rank_sim.py --views 32 --worlds 1,2,4,8 --steps 4
run ranksim64 200 python tools/rank_sim.py --views 64 --worlds 1,8 --steps 2
