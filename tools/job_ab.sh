#!/usr/bin/env bash
# One-off A/B job: GPU steps in order, each under its own time limit; stops at the first failure.
set -u
mkdir -p gpurun_out
run() { local name=$1 secs=$2; shift 2; echo "=== $name" >> gpurun_out/job.log; timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc" >> gpurun_out/job.log; [ $rc -eq 0 ] || exit $rc; }
T="--timeout 600 --timeout-method thread"
case ${1:-} in
  split)
    run split_test 600 python -u -m pytest tests/test_baseline_shapes_gpu.py -x -q -m gpu -k "split or reloc" $T
    run kreloc 300 python tools/kbench.py attn
    run parity_split 900 env SR_RELOC_SPLIT=1 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "c3 or c2" $T
    for i in 1 2; do
      run bench_rs0_$i 400 env SR_RELOC_SPLIT=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
      run bench_rs1_$i 400 env SR_RELOC_SPLIT=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
    done ;;
  conc)
    for i in 1 2; do
      run bench_cs0_$i 400 env SR_CONCURRENT_STACKS=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
      run bench_cs1_$i 400 env SR_CONCURRENT_STACKS=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
    done
    run parity_conc 900 env SR_CONCURRENT_STACKS=1 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "c3 or c2" $T ;;
  pair)
    run pair_test 600 python -u -m pytest tests/test_baseline_shapes_gpu.py -x -q -m gpu -k "pair or split" $T
    run kpair 300 python tools/kbench.py attn_pair
    run parity_pair 900 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "c3 or c2" $T
    for i in 1 2; do
      run bench_pr0_$i 400 env SR_ATTN_PAIR=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
      run bench_pr1_$i 400 env SR_ATTN_PAIR=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
    done ;;
  group)
    run group_test 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_baseline_shapes_gpu.py -x -q -m gpu -k "group or pair" $T
    run parity_group 900 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu -k "c3 or c2" $T
    for i in 1 2; do
      run bench_gg0_$i 400 env SR_GEMM_GROUP=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
      run bench_gg1_$i 400 env SR_GEMM_GROUP=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
    done ;;
  wgrad)
    run wgrad_test 600 python -u -m pytest tests/test_train_kernels_gpu.py tests/test_train_block_gpu.py -x -q -m gpu $T
    for i in 1 2; do
      run ktrain_w0_$i 600 env SR_WGRAD256=0 python tools/kbench.py train
      run ktrain_w1_$i 600 env SR_WGRAD256=1 python tools/kbench.py train
    done ;;
  evidence)
    run pmc_pair1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_pair1 -o run --output-format csv -- python3 tools/kbench.py attn_pair
    run pmc_pair2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_pair2 -o run --output-format csv -- python3 tools/kbench.py attn_pair
    run ktrain 900 python tools/kbench.py train
    run prof_train 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 tools/kbench.py train ;;
  smallm)
    run smallm_test 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_layers_gpu.py -x -q -m gpu -k "gemm or camera or block" $T
    run parity_smallm 900 python -u -m pytest tests/test_parity_gpu.py -x -q -m gpu $T
    for i in 1 2; do
      run bench_sm0_$i 400 env SR_GEMM_SMALLM=0 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
      run bench_sm1_$i 400 env SR_GEMM_SMALLM=1 python bench.py --steps 4 --warmup 1 --no-cpu-baseline
    done
    run ktrain 900 python tools/kbench.py train ;;
  final)
    run gputests 1200 python -u -m pytest tests -x -q -m gpu $T
    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    run bench 600 python bench.py
    run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing
    run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing
    run pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing
    run pmc_pair1 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_pair1 -o run --output-format csv -- python3 tools/kbench.py attn_pair
    run pmc_pair2 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/pmc_pair2 -o run --output-format csv -- python3 tools/kbench.py attn_pair
    run prof_train 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 tools/kbench.py train ;;
  lnb)
    run lnb_test 600 python -u -m pytest tests/test_train_kernels_gpu.py tests/test_train_block_gpu.py -x -q -m gpu $T
    for i in 1 2; do
      run ktrain_lnb0_$i 600 env SFM_AMD_LIB=variants/libsfm_lnb0.so python tools/kbench.py train
      run ktrain_lnb1_$i 600 python tools/kbench.py train
    done
    run prof_lnb1 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lnb1 -o run --output-format csv -- python3 tools/kbench.py train
    run prof_lnb0 900 env SFM_AMD_LIB=variants/libsfm_lnb0.so rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lnb0 -o run --output-format csv -- python3 tools/kbench.py train
    run c4_golden 900 python -u -m pytest tests/test_c4_golden_gpu.py -x -q -m gpu $T ;;
  *) echo "unknown job ${1:-}"; exit 2 ;;
esac
