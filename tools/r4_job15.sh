#!/usr/bin/env bash
# round-4 GPU job 15: which attention waves leave the hand-scheduled sweep at qk-norm gains 1-4
set -u
mkdir -p gpurun_out
timeout -k 10 400 python tools/sweep_stats.py --gains 1,2,3,4 > gpurun_out/sweep_stats.log 2>&1
rc=$?; tail -n 5 gpurun_out/sweep_stats.log; exit $rc
