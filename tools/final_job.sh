#!/usr/bin/env bash
# final validation of a round (tools/final_job.sh A|B|C|D).  A = every GPU test but the multi-rank ones, B = the multi-rank tests +
# smoke, C = default bench (cpu baseline, extras) + rocprofv3 kernel stats (1 and 3 steps: the
# steady-state counts) + FETCH_SIZE / WRITE_SIZE PMC passes, D = training kernel stats + an unprofiled training step, E = the per-rank rehearsal (tools/rank_sim.py).
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 3 | cut -c1-300
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
T="--timeout 600 --timeout-method thread"
NB="--no-cpu-baseline --no-kernel-timing --extras none"
case ${1:-} in
  A) run f_tests_a 1100 python -u -m pytest tests -q -m gpu $T \
       --ignore tests/test_dist_gpu.py --ignore tests/test_train_step_gpu.py --ignore tests/test_c4_golden_gpu.py ;;
  B) run f_tests_b 1000 python -u -m pytest tests/test_dist_gpu.py tests/test_train_step_gpu.py tests/test_c4_golden_gpu.py -q -m gpu $T
     run f_smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
  C) run f_bench 500 python bench.py
     run f_prof_s1 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f_prof_s1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 $NB
     run f_prof_s3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f_prof_s3 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 $NB
     run f_pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/f_pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 $NB
     run f_pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/f_pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 $NB ;;
  D) run f_prof_train 500 rocprofv3 --kernel-trace --stats -d gpurun_out/f_prof_train -o run --output-format csv -- python3 tools/kbench.py train
     run f_ktrain 500 python tools/kbench.py train ;;
  E) run f_rank_sim 900 python tools/rank_sim.py --worlds 1,2,4,8 --steps 5 ;;
  *) echo "usage: $0 A|B|C|D|E"; exit 2 ;;
esac
