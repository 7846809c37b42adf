#!/usr/bin/env bash
# round-5 GPU job 26: SQ counters of the attention backward, compiled vs asm sweeps (kbench
# attn_bwd runs both: the kernels have distinct names), two passes of <= 8 SQ counters each
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp SR_BWD_RELOC=0
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/j26_pmc1 -o run --output-format csv -- python3 tools/kbench.py attn_bwd > gpurun_out/j26_pmc1.log 2>&1 || { echo "pmc1 failed"; tail -5 gpurun_out/j26_pmc1.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/j26_pmc2 -o run --output-format csv -- python3 tools/kbench.py attn_bwd > gpurun_out/j26_pmc2.log 2>&1 || { echo "pmc2 failed"; tail -5 gpurun_out/j26_pmc2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/j26_pmc1 gpurun_out/j26_pmc2 attn_bwd | tee gpurun_out/j26_pmc_bwd.txt
