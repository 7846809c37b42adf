# L2 (TCC) write-path counters of the GEMM kernels (kbench gemm shapes), one pass per counter group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum" \
           "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum" \
           "TCC_NORMAL_WRITEBACK_sum TCC_NORMAL_EVICT_sum TCC_BUSY_avr TCC_IB_STALL_sum" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc_tcc$i -o run --output-format csv -- \
    python3 tools/kbench.py gemm > gpurun_out/pmc_tcc$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_tcc$i.log; exit 1; }
  echo "pass $i ok"
done
