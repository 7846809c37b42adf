#!/usr/bin/env bash
# round-5 GPU job 25: the concatenated-items dK/dV asm sweep (SR_ATTN_BWD_CAT=1): tests, kbench
# attn_bwd (global / frame / reloc), training A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|attn_bwd|ms/step|concatenated" "gpurun_out/$name.log" | cut -c1-160 | tail -n 24
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j25_tests 300 python -u -m pytest tests/test_attn_bwd_gpu.py -x -q -s -m gpu --timeout 120 --timeout-method thread
run j25_kbwd 400 python tools/kbench.py attn_bwd
run j25_train0 400 python tools/kbench.py train
SR_ATTN_BWD_CAT=1 run j25_train1 400 python tools/kbench.py train
