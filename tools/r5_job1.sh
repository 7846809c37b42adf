#!/usr/bin/env bash
# round-5 GPU job 1: the ABI 1.0 changes (q rounded once: sr_gemm_epi.q_scale + sr_attn_desc.q_scaled,
# key_norm2, sized colsum workspace) -- the whole GPU suite with the measured parity errors printed,
# then a quick bench A/B of the q convention.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|views/s" "gpurun_out/$name.log" | cut -c1-300 | tail -n 6
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j1_tests 1100 python -u -m pytest tests --maxfail=15 -q -s -m gpu --timeout 600 --timeout-method thread
run j1_bench_qs1 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras ''
SR_Q_PRESCALE=0 run j1_bench_qs0 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras ''
run j1_bench_qs1b 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline --extras ''
