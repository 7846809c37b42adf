#!/usr/bin/env bash
# round-4 final validation: A = every GPU test + smoke; B = default bench (cpu baseline, extras),
# rocprofv3 kernel stats, FETCH_SIZE / WRITE_SIZE PMC passes, training kernel stats.
set -u
mkdir -p gpurun_out
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
T="--timeout 600 --timeout-method thread"
case ${1:-} in
  A)
    run gputests 1000 python -u -m pytest tests -x -q -m gpu $T
    run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
  B)
    run bench 500 python bench.py
    run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
    run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
    run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
    run prof_train 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- \
      python3 tools/kbench.py train ;;
  C)
    run cpu_full 1150 python tools/cpu_full.py ;;
  *) echo "usage: $0 A|B|C"; exit 2 ;;
esac
