#!/usr/bin/env bash
# round-5 GPU job 6: the pair launch of this round's library against round 4's final build
# (ab/libsfm_r04.so, git 70ba086, the same sources' kernels), same box, interleaved; the attention
# key-scan and production-shape tests.
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|attn pair|key scan" "gpurun_out/$name.log" | cut -c1-200 | tail -n 8
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j6_tests 600 python -u -m pytest tests/test_baseline_shapes_gpu.py -q -s -m gpu -k "key_scan or frame_attention or global_attention or reloc_attention" --timeout 300 --timeout-method thread
for i in 1 2 3; do
  SFM_AMD_LIB=ab/libsfm_r04.so run j6_pair_r04_$i 200 python tools/kbench.py attn_pair
  run j6_pair_r05_$i 200 python tools/kbench.py attn_pair
done
