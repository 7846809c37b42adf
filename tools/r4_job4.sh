#!/usr/bin/env bash
# round-4 GPU job 4: GEMM last-round tail split (SR_GEMM_TAIL) tests + A/B on the C3 bench and
# the per-rank rehearsal
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
run ttail 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -s -m gpu --timeout 250 --timeout-method thread -k "gemm_tail or gemm_group or gemm256"
run b_t0a 300 env SR_GEMM_TAIL=0 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run b_t1a 300 env SR_GEMM_TAIL=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run b_t0b 300 env SR_GEMM_TAIL=0 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run b_t1b 300 env SR_GEMM_TAIL=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none
run rs_t1 200 env SR_GEMM_TAIL=1 python tools/rank_sim.py --views 32 --worlds 2,4,8 --steps 4
