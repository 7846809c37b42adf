#!/usr/bin/env bash
# round-5 GPU job 17: where the hand-scheduled dK/dV sweep's time goes -- timing-only ablation
# builds of tools/gen_attn_bwd_pipe.py (ab/libsfm_pv_*.so: no barrier / no DMA / no VALU / no LDS
# reads / no waits / MFMAs only) and two schedule knobs, each timed by kbench attn_bwd (asm arm)
set -u
mkdir -p gpurun_out
for v in base nobar nodma novalu noread nowait mfmaonly lead0 rd55 base; do
  echo "== $v"
  SFM_AMD_LIB=ab/libsfm_pv_$v.so SR_BWD_AB=pipe timeout -k 10 120 python3 tools/kbench.py attn_bwd > gpurun_out/j17_$v.log 2>&1 || { echo "failed $v"; tail -20 gpurun_out/j17_$v.log; exit 1; }
  grep attn_bwd gpurun_out/j17_$v.log
done
