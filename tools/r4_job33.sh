#!/usr/bin/env bash
# round-4 GPU job 33: PMC passes on the final tree's pair launch (kbench attn_pair), two separate
# counter sets (8 SQ each; no trace domains), summarised by tools/pmc_summary.py
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/j33_pmc1 -o run --output-format csv -- python3 tools/kbench.py attn_pair > gpurun_out/j33_pmc1.log 2>&1 || { echo "pmc1 failed"; tail -5 gpurun_out/j33_pmc1.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/j33_pmc2 -o run --output-format csv -- python3 tools/kbench.py attn_pair > gpurun_out/j33_pmc2.log 2>&1 || { echo "pmc2 failed"; tail -5 gpurun_out/j33_pmc2.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/j33_pmc1 gpurun_out/j33_pmc2 attn > gpurun_out/j33_pmc_pair.txt 2>&1
grep -h "attn pair" gpurun_out/j33_pmc1.log gpurun_out/j33_pmc2.log >> gpurun_out/j33_pmc_pair.txt
cat gpurun_out/j33_pmc_pair.txt
