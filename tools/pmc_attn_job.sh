set -u
mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for cfg in 0 3; do
  for p in 1 2; do
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    SR_ATTN_CFG=$cfg timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/pmc_c${cfg}_$p -o run --output-format csv -- python3 tools/kbench.py attn > gpurun_out/pmc_c${cfg}_$p.log 2>&1 || { echo "fail cfg=$cfg p=$p"; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_c${cfg}_1 gpurun_out/pmc_c${cfg}_2 attn
done
