#!/usr/bin/env bash
# round-5 GPU job 13: grouped tails at every size (SR_GROUP_TAILS=2) on one GPU (the paired global +
# reloc tails at 43,968 rows each) against the default, interleaved.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"" "gpurun_out/$name.log" | cut -c1-130 | tail -n 3
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
SR_GROUP_TAILS=2 run j13_tests 400 python -u -m pytest tests/test_parity_gpu.py -q -s -m gpu -k "c3 or n8" --timeout 300 --timeout-method thread
for i in 1 2 3; do
  run j13_bench_g1_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  SR_GROUP_TAILS=2 run j13_bench_g2_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
