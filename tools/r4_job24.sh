#!/usr/bin/env bash
# round-4 GPU job 24: training-step kernel stats (rocprofv3) on the current tree
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/j24_prof_train -o run --output-format csv -- \
  python3 tools/kbench.py train > gpurun_out/j24_prof_train.log 2>&1
rc=$?; tail -n 30 gpurun_out/j24_prof_train.log | grep -v "^W2026\|^E2026"; exit $rc
