#!/usr/bin/env bash
# round-5 GPU job 2: tightened parity bounds (parity + tail-split tests), the q-convention bench A/B,
# the default bench with the C5 qkv / qk extras, camera-GEMM split sweep, steady-state launch counts.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|\"value\"" "gpurun_out/$name.log" | cut -c1-300 | tail -n 4
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j2_tests 900 python -u -m pytest tests/test_parity_gpu.py tests/test_kernels_gpu.py -k "parity or full or small or block_kats or tail_split" -q -s -m gpu --timeout 600 --timeout-method thread
for i in 1 2; do
  run j2_bench_qs1_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
  SR_Q_PRESCALE=0 run j2_bench_qs0_$i 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras none
done
run j2_kcam 300 python tools/kbench.py gemm_cam
run j2_bench_full 600 python bench.py --no-cpu-baseline
run j2_prof_s1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/j2_prof_s1 -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
run j2_prof_s3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/j2_prof_s3 -o run --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
