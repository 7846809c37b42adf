#!/usr/bin/env bash
# round-5 GPU job 9: the MLP in MALL-sized row chunks (SR_MLP_CHUNK=16384): C3 golden with it, then
# the step A/B, interleaved.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"" "gpurun_out/$name.log" | cut -c1-160 | tail -n 4
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
SR_MLP_CHUNK=16384 run j9_tests 400 python -u -m pytest tests/test_parity_gpu.py -q -s -m gpu -k "c3 or n8" --timeout 300 --timeout-method thread
for i in 1 2 3; do
  run j9_bench_c0_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  SR_MLP_CHUNK=16384 run j9_bench_c1_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
