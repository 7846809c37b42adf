#!/usr/bin/env bash
# Run named GPU steps in order, each under its own time limit, logging to gpurun_out/.
# Stops at the first step that fails in any way (a Python-level HIP fault exits 1 too, so
# no later step may touch the GPU after it).
#   tools/gpu_job.sh kernels parity smoke bench [prof]
set -u
mkdir -p gpurun_out
status=0
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/job.log
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 6
  if [ "$rc" -ne 0 ]; then echo "=== $name failed (rc=$rc): stopping"; exit "$rc"; fi
}
for step in "$@"; do
  case $step in
    kernels) run kernels 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu ;;
    parity)  run parity 900 python -m pytest tests/test_parity_gpu.py -x -q -m gpu ;;
    gputests) run gputests 1200 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} ;;
    newtests) run newtests 900 python -u -m pytest tests/test_baseline_shapes_gpu.py tests/test_layers_gpu.py \
                tests/test_demo_entry_gpu.py tests/test_parity_gpu.py tests/test_train_graph_gpu.py -x -v -m gpu \
                --timeout 600 --timeout-method thread ;;
    disttests) run disttests 900 python -u -m pytest tests/test_dist_gpu.py tests/test_baseline_shapes_gpu.py -x -v -m gpu \
                --timeout 600 --timeout-method thread ;;
    gemm_tests) run gemm_tests 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k gemm ;;
    attn_tests) run attn_tests 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k attention ;;
    attn_tests1) run attn_tests1 300 env SR_ATTN_CFG=1 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k attention ;;
    kattn_cfg1) run kattn_cfg1 300 env SR_ATTN_CFG=1 python tools/kbench.py attn ;;
    kattn_cfgs) for i in 1 2; do
                  for c in 0 1 2; do run kattn_cfg${c}_$i 300 env SR_ATTN_CFG=$c SR_KB_STATIC=1 python tools/kbench.py attn || exit 1; done
                done ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 600 python bench.py ;;
    benchq)  run benchq 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    bench_c2) run bench_c2 400 python bench.py --views 8 --no-cpu-baseline ;;
    bench64) run bench64 600 python bench.py --views 64 --steps 5 --warmup 2 --no-cpu-baseline ;;
    prof64)  run prof64 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- \
               python3 bench.py --views 64 --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing ;;
    bench_extra) run bench_extra 600 python bench.py --steps 4 --warmup 1 --no-cpu-baseline --extra-c5 qkv ;;
    bench_c5) run bench_c5 600 python bench.py --views 128 --steps 2 --warmup 1 --no-cpu-baseline ;;
    bench_c5q) run bench_c5q 600 python bench.py --views 128 --steps 2 --warmup 1 --no-cpu-baseline --fp8-global qkv ;;
    kbench)  run kbench 300 python tools/kbench.py ;;
    kgemm)   run kgemm 300 python tools/kbench.py gemm ln ;;
    kgemm_128) for i in 1 2; do
                run kgemm_256_$i 300 python tools/kbench.py gemm || exit 1
                run kgemm_128_$i 300 env SR_GEMM_NO256=1 python tools/kbench.py gemm || exit 1
              done ;;
    reloc_split_ab) for i in 1 2; do
                run bench_rs0_$i 400 env SR_RELOC_SPLIT=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline || exit 1
                run bench_rs1_$i 400 env SR_RELOC_SPLIT=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline || exit 1
              done ;;
    parity_c3) run parity_c3 900 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu -k "c3 or c2" --timeout 600 --timeout-method thread ;;
    kgemm_reg) run kgemm_reg 300 env SR_GEMM_REG_EPI=1 python tools/kbench.py gemm ;;
    kdpt)    run kdpt 600 python tools/kbench.py dpt ;;
    kreloc)  run kreloc 600 python tools/kbench.py reloc ;;
    kio)     run kio 300 python tools/kbench.py io ;;
    io_tests) run io_tests 600 python -m pytest tests/test_io_gpu.py -q -x ;;
    kattn)   run kattn 300 python tools/kbench.py attn ;;
    dbg_pipe) run dbg_pipe 300 env SR_ATTN_PIPE=1 python tools/dbg_attn_pipe.py 1024 8192 8256 16384 16448 16512 16576 43968 ;;
    kattn_ab) run kattn_ab0 300 env SR_ATTN_PIPE=0 SR_KB_STATIC=1 python tools/kbench.py attn && \
              run kattn_ab1 300 env SR_ATTN_PIPE=1 SR_KB_STATIC=1 python tools/kbench.py attn && \
              run kattn_ab2 300 env SR_ATTN_PIPE=0 SR_KB_STATIC=1 python tools/kbench.py attn && \
              run kattn_ab3 300 env SR_ATTN_PIPE=1 SR_KB_STATIC=1 python tools/kbench.py attn ;;
    attn_pipe_tests) run attn_pipe_tests 900 env SR_ATTN_PIPE=1 python -u -m pytest tests/test_baseline_shapes_gpu.py \
              tests/test_kernels_gpu.py -x -q -m gpu -k "attention or attn" --timeout 600 --timeout-method thread ;;
    attn_shape_tests) run attn_shape_tests 900 python -u -m pytest tests/test_baseline_shapes_gpu.py tests/test_kernels_gpu.py \
              -x -q -m gpu -k "attention or attn" --timeout 600 --timeout-method thread ;;
    c4test)  run c4test 900 python -u -m pytest tests/test_c4_golden_gpu.py -x -v -s -m gpu --timeout 900 --timeout-method thread ;;
    fp8test) run fp8test 900 python -u -m pytest tests/test_parity_gpu.py -x -v -s -m gpu -k fp8 --timeout 600 --timeout-method thread ;;
    kattn_var) for i in 1 2; do
                 run kattn_v0_$i 300 env SR_ATTN_PIPE=0 SR_KB_STATIC=1 python tools/kbench.py attn || exit 1
                 for v in $PIPE_VARIANTS; do
                   run kattn_${v}_$i 300 env SFM_AMD_LIB=variants/libsfm_$v.so SR_ATTN_PIPE=1 SR_KB_STATIC=1 python tools/kbench.py attn || exit 1
                 done
                 run kattn_main_$i 300 env SR_ATTN_PIPE=1 SR_KB_STATIC=1 python tools/kbench.py attn || exit 1
               done ;;
    dbg_var) for v in $PIPE_VARIANTS; do
               run dbg_$v 300 env SFM_AMD_LIB=variants/libsfm_$v.so SR_ATTN_PIPE=1 python tools/dbg_attn_pipe.py 8192 8256 16384 16448 43968 || exit 1
             done ;;
    kattn_seg) for i in 1 2; do
                 run kattn_seg0_$i 300 env SR_ATTN_PIPE_SEG=0 SR_KB_STATIC=1 python tools/kbench.py attn || exit 1
                 run kattn_seg1_$i 300 env SR_ATTN_PIPE_SEG=1 SR_KB_STATIC=1 python tools/kbench.py attn || exit 1
               done ;;
    kfdiag)  run kfdiag0 300 python tools/kbench.py attn_frame_diag && \
             run kfdiag1 300 env SR_ATTN_PIPE_SEG=1 python tools/kbench.py attn_frame_diag ;;
    parity_split) run parity_split 900 env SR_RELOC_SPLIT=1 python -u -m pytest tests/test_parity_gpu.py -x -v -m gpu -k "c3 or c2" --timeout 600 --timeout-method thread ;;
    resln_ab) for i in 1 2; do
                run bench_rl0_$i 400 env SR_FUSED_RESID_LN=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline || exit 1
                run bench_rl1_$i 400 env SR_FUSED_RESID_LN=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline || exit 1
              done ;;
    kln)     run kln 300 python tools/kbench.py ln ;;
    kb_ab)   for i in 1 2; do  # kbench modes $AB_KB: ablib/libsfm_${AB_NAME}.so (an earlier build) against the committed one
               run kb_${AB_NAME}_$i 300 env SFM_AMD_LIB=ablib/libsfm_${AB_NAME}.so python tools/kbench.py $AB_KB || exit 1
               run kb_new_$i 300 python tools/kbench.py $AB_KB || exit 1
             done ;;
    bench_ab) for i in 1 2; do
               run bench_${AB_NAME}_$i 400 env SFM_AMD_LIB=ablib/libsfm_${AB_NAME}.so python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
               run bench_new_$i 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
             done ;;
    kgemm_var) for i in 1 2; do
                 run kgemm_v0_$i 300 python tools/kbench.py gemm || exit 1
                 for v in $GEMM_VARIANTS; do
                   run kgemm_${v}_$i 300 env SFM_AMD_LIB=variants/libsfm_$v.so python tools/kbench.py gemm || exit 1
                 done
               done ;;
    kattn4)  run kattn4 300 env SR_ATTN_WAVES=4 python tools/kbench.py attn ;;
    kattn2)  run kattn2 300 env SR_ATTN_WAVES=2 python tools/kbench.py attn ;;
    prof)    run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
               python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing ;;
    pmc_fetch) run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
               python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing ;;
    pmc_fetch_c5q) run pmc_fetch_c5q 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_c5q -o run --output-format csv -- \
               python3 bench.py --views 128 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --fp8-global qkv ;;
    pmc_write_c5q) run pmc_write_c5q 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_c5q -o run --output-format csv -- \
               python3 bench.py --views 128 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing --fp8-global qkv ;;
    pmc_write) run pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
               python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing ;;
    pmc_gemm1) run pmc_gemm1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_gemm1 -o run --output-format csv -- python3 tools/kbench.py gemm ;;
    pmc_gemm2) run pmc_gemm2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_gemm2 -o run --output-format csv -- python3 tools/kbench.py gemm ;;
    pmc_gemm3) run pmc_gemm3 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL TA_BUSY_avr GRBM_GUI_ACTIVE -d gpurun_out/pmc_gemm3 -o run --output-format csv -- python3 tools/kbench.py gemm ;;
    counters) run counters 120 rocprofv3 -L ;;
    pmc_attn1) run pmc_attn1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_attn1 -o run --output-format csv -- python3 tools/kbench.py attn gemm ;;
    pmc_attn2) run pmc_attn2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn2 -o run --output-format csv -- python3 tools/kbench.py attn gemm ;;
    pmc_attnp1) run pmc_attnp1 300 env SR_ATTN_PIPE=1 SR_KB_STATIC=1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_attnp1 -o run --output-format csv -- python3 tools/kbench.py attn ;;
    pmc_attnp2) run pmc_attnp2 300 env SR_ATTN_PIPE=1 SR_KB_STATIC=1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_attnp2 -o run --output-format csv -- python3 tools/kbench.py attn ;;
    pmc_attnp3) run pmc_attnp3 300 env SR_ATTN_PIPE=1 SR_KB_STATIC=1 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc_attnp3 -o run --output-format csv -- python3 tools/kbench.py attn ;;
    pmc_attn0) run pmc_attn0 300 env SR_ATTN_PIPE=0 SR_KB_STATIC=1 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_attn0 -o run --output-format csv -- python3 tools/kbench.py attn ;;
    kattnb)  run kattnb 300 python tools/kbench.py attn_bwd ;;
    ktrain)  run ktrain 900 python tools/kbench.py train ;;
    prof_train) run prof_train 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- \
               python3 tools/kbench.py train ;;
    pmc_bwd1) run pmc_bwd1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_bwd1 -o run --output-format csv -- python3 tools/kbench.py attn_bwd ;;
    pmc_bwd2) run pmc_bwd2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_bwd2 -o run --output-format csv -- python3 tools/kbench.py attn_bwd ;;
    tests_a) run tests_a 1100 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread \
               --ignore tests/test_dist_gpu.py --ignore tests/test_train_step_gpu.py --ignore tests/test_c4_golden_gpu.py ;;
    tests_b) run tests_b 1000 python -u -m pytest tests/test_dist_gpu.py tests/test_train_step_gpu.py \
               tests/test_c4_golden_gpu.py -q -m gpu --timeout 600 --timeout-method thread ;;
    # 256x256 GEMM tile order A/B (SR_GEMM_GROUP_M = g row tiles per group; 1 = row-major): kbench
    # timings, then per-launch fetch / clock from one FETCH_SIZE + GRBM_GUI_ACTIVE pass per order
    raster) for g in ${RASTER_GROUPS:-1 4 8 16}; do
              run kgemm_g${g} 300 env SR_GEMM_GROUP_M=$g python tools/kbench.py gemm gemm_qkv || exit 1
            done
            for g in ${RASTER_GROUPS:-1 4 8 16}; do
              run pmc_raster_g${g} 300 env SR_GEMM_GROUP_M=$g rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
                -d gpurun_out/pmc_raster_g${g} -o run --output-format csv -- python3 tools/kbench.py gemm || exit 1
              python tools/pmc_dispatch.py gpurun_out/pmc_raster_g${g} gemm > gpurun_out/pmc_raster_g${g}.txt
            done ;;
    gemm_tests2) run gemm_tests2 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 300 --timeout-method thread ;;
    kresid)  run kresid 300 python tools/kbench.py gemm_resid gemm ;;
    train_tests) run train_tests 1100 python -u -m pytest tests/test_train_graph_gpu.py tests/test_train_kernels_gpu.py \
               tests/test_train_block_gpu.py tests/test_attn_bwd_gpu.py tests/test_c4_golden_gpu.py tests/test_train_step_gpu.py \
               -x -q -m gpu --timeout 900 --timeout-method thread ;;
    resid_ab) for i in 1 2; do
                run bench_rl0_$i 400 env SR_GEMM_RESID_LDS=0 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
                run bench_rl1_$i 400 env SR_GEMM_RESID_LDS=1 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
              done ;;
    pair_tests) run pair_tests 600 python -u -m pytest tests/test_baseline_shapes_gpu.py -x -q -m gpu -k "pair or dma_base or qk_gain" \
               --timeout 300 --timeout-method thread ;;
    kpair)   run kpair 300 python tools/kbench.py attn_pair ;;
    kqk)     run kqk 300 python tools/kbench.py qk_bwd ;;
    resid_modes) for i in ${RM_RUNS:-1 2}; do  # proj -> LN2 fusion (SR_FUSED_RESID_LN) x fc2 -> next LN1 (SR_DEFER_RESID)
                   for m in ${RM_MODES:-00 10 01 11}; do
                     run bench_rm${m}_$i 400 env SR_FUSED_RESID_LN=${m:0:1} SR_DEFER_RESID=${m:1:1} python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
                   done
                 done ;;
    lib_ab)  for i in 1 2; do  # the committed build against ablib/libsfm_${AB_NAME}.so (an earlier build)
               run kln_${AB_NAME}_$i 300 env SFM_AMD_LIB=ablib/libsfm_${AB_NAME}.so python tools/kbench.py ln || exit 1
               run kln_new_$i 300 python tools/kbench.py ln || exit 1
               run bench_${AB_NAME}_$i 400 env SFM_AMD_LIB=ablib/libsfm_${AB_NAME}.so python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
               run bench_new_$i 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --extras none || exit 1
             done ;;
    train_ab) for i in 1 2; do
                for m in ${TRAIN_AB_MODES:-0 3}; do
                  run ktrain_cs${m}_$i 600 env SR_TRAIN_BIAS_COLSUM=$m python tools/kbench.py train || exit 1
                done
              done ;;
    pmc_pair) run pmc_pair1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_pair1 -o run --output-format csv -- python3 tools/kbench.py attn_pair && \
              run pmc_pair2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_pair2 -o run --output-format csv -- python3 tools/kbench.py attn_pair && \
              run pmc_pair3 300 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d gpurun_out/pmc_pair3 -o run --output-format csv -- python3 tools/kbench.py attn_pair ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit $status
