#!/usr/bin/env bash
# round-4 GPU job 18: per-layer window diagnostics of the global attention at qk-gain 4
set -u
mkdir -p gpurun_out
timeout -k 10 400 python tools/sweep_stats.py --gains 4 --box auto --diag > gpurun_out/j18_sweep.log 2>&1
rc=$?; tail -c 3000 gpurun_out/j18_sweep.log; exit $rc
