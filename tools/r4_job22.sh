#!/usr/bin/env bash
# round-4 GPU job 22: the key box reduction at 1024 threads, <= 512 partials: parity, its cost
# at qk-gain 4 (rocprofv3 stats), the headline at g = 4 and g = 1
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -n 4 "gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; exit $rc; fi
}
run j22_tests 420 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
    -k "key_box or value_window or qk_gain" tests/test_kernels_gpu.py tests/test_baseline_shapes_gpu.py
export TMPDIR=/tmp
run j22_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/j22_prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --extras none --qk-gain 4
run j22_bench_g4 300 python bench.py --steps 5 --warmup 2 --extras none --qk-gain 4
run j22_bench_g1 300 python bench.py --steps 5 --warmup 2 --extras none --qk-gain 1
