#!/usr/bin/env bash
# round-4 GPU job 14: every GPU test + smoke + default bench on the final tree, then the headline at qk-norm gains 1-4
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
run gputests 800 python -u -m pytest tests --maxfail 5 -q -m gpu $T
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 400 python bench.py
for g in 1 2 3 4; do
  run gain$g 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none --qk-gain $g
done
