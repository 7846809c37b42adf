#!/usr/bin/env bash
# round-5 GPU job 20: training-step kernel profile with the hand-scheduled backward sweeps on
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/j20_prof -o run --output-format csv -- python3 tools/kbench.py train > gpurun_out/j20_train.log 2>&1 || { echo "failed"; tail -30 gpurun_out/j20_train.log; exit 1; }
grep "train:" gpurun_out/j20_train.log
cp gpurun_out/j20_prof/run_kernel_stats.csv gpurun_out/j20_train_kernel_stats.csv
python3 tools/train_breakdown.py gpurun_out/j20_train_kernel_stats.csv 4 | tee gpurun_out/j20_train_breakdown.txt
