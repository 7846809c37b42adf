# GEMM tuning job: GEMM tests on the shipped library and on each variant, then interleaved
# kbench gemm rounds (shipped vs variants), then hipBLASLt kernel names under rocprofv3.
#   VARS="STAG PRIO4" bash tools/ab_gemm_var.sh
set -o pipefail
mkdir -p gpurun_out
for v in - $VARS; do
  lib=""; [ "$v" = "-" ] || lib=self-supervise-sfm_amd/variants/lib_$v.so
  case " NOEPI SAMEOUT $NOTEST " in *" $v "*) continue;; esac
  SFM_AMD_LIB=$lib timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k gemm > gpurun_out/gemm_tests_$v.log 2>&1 || { tail -20 gpurun_out/gemm_tests_$v.log; exit 1; }
  echo "tests $v: $(tail -1 gpurun_out/gemm_tests_$v.log)"
done
for i in 1 2; do
  for v in - $VARS; do
    lib=""; [ "$v" = "-" ] || lib=self-supervise-sfm_amd/variants/lib_$v.so
    echo "== $v"; SFM_AMD_LIB=$lib timeout -k 10 200 python tools/kbench.py gemm 2>/dev/null | grep -v amdgpu || exit 1
  done
done
