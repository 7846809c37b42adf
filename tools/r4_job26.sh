#!/usr/bin/env bash
# round-4 GPU job 26: the block GEMMs with the 256x256 kernel vs the 128x128 kernel only
# (SR_GEMM_NO256), C3 rows -- does the two-workgroups-per-CU overlap pay for the fp32 residual
# epilogue of proj (K = 1024)?
set -u
mkdir -p gpurun_out
timeout -k 10 200 python tools/kbench.py gemm gemm_k > gpurun_out/j26_gemm256.log 2>&1 || exit 1
SR_GEMM_NO256=1 timeout -k 10 200 python tools/kbench.py gemm gemm_k > gpurun_out/j26_gemm128.log 2>&1 || exit 1
timeout -k 10 200 python tools/kbench.py gemm > gpurun_out/j26_gemm256b.log 2>&1
rc=$?; grep -h "gemm" gpurun_out/j26_gemm256.log gpurun_out/j26_gemm128.log gpurun_out/j26_gemm256b.log; exit $rc
