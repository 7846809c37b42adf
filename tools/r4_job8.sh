#!/usr/bin/env bash
# round-4 GPU job 8: key-split test, smoke, default bench + rocprof + PMC traffic passes,
# attention-backward counters
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
run keysplit 200 python -u -m pytest tests/test_baseline_shapes_gpu.py -q -s -m gpu -k key_split $T
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
run bench 500 python bench.py
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --extras none
run pmc_bwd1 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_bwd1 -o run --output-format csv -- python3 tools/kbench.py attn_bwd
run pmc_bwd2 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_bwd2 -o run --output-format csv -- python3 tools/kbench.py attn_bwd
