#!/usr/bin/env bash
# round-5 GPU job 16: per-kernel times of the attention backward (kbench attn_bwd runs both the
# compiled and the hand-scheduled dK/dV sweep; the kernels have distinct names)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/j16_prof -o run --output-format csv -- python3 tools/kbench.py attn_bwd > gpurun_out/j16_kbwd.log 2>&1 || { echo "failed"; tail -30 gpurun_out/j16_kbwd.log; exit 1; }
grep attn_bwd gpurun_out/j16_kbwd.log
f=$(find gpurun_out/j16_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/j16_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/j16_stats.csv')):
    if 'attn' in r['Name']: print(r['Name'][:90], r['Calls'], r['AverageNs'], r['MinNs'], r['MaxNs'])
"
