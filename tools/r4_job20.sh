#!/usr/bin/env bash
# round-4 GPU job 20: the key / value box passes' cost at qk-gain 4 (rocprofv3 stats) and the
# frame / reloc attention with and without them
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/j20_prof -o j20 -- python3 bench.py --steps 3 --warmup 1 --extras none --qk-gain 4 > gpurun_out/j20_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/j20_prof.log; exit 1; }
export SR_ATTN_KEY_BOX=0
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --extras none --qk-gain 4 > gpurun_out/j20_bench_g4_nobox.log 2>&1
rc=$?; tail -c 600 gpurun_out/j20_bench_g4_nobox.log; find gpurun_out/j20_prof -name "*kernel_stats.csv" | head; exit $rc
