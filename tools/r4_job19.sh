#!/usr/bin/env bash
# round-4 GPU job 19: the scanned key norm (norm2_out) with the key and value boxes -- parity, which waves stay
# on the hand-scheduled sweep at qk-gains 1 and 4 with and without it, and the headline at g = 4 / 1
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 6 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; exit $rc; fi
}
run j19_tests 420 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
    -k "key_box or value_window or qk_gain" tests/test_kernels_gpu.py tests/test_baseline_shapes_gpu.py
run j19_sweep 500 python tools/sweep_stats.py --gains 4,4.5 --box auto
run j19_bench_g4 300 python bench.py --steps 5 --warmup 2 --extras none --qk-gain 4
run j19_bench_g1 300 python bench.py --steps 5 --warmup 2 --extras none --qk-gain 1
