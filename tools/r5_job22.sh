#!/usr/bin/env bash
# round-5 GPU job 22: the dQ asm sweep over two key segments (reloc), the shared-key dK/dV item
# split (SR_ATTN_BWD_QSPLIT): tests, kbench attn_bwd with the reloc shape, training A/B
set -u
mkdir -p gpurun_out
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  grep -E "passed|failed|Error|attn_bwd|ms/step" "gpurun_out/$name.log" | cut -c1-160 | tail -n 20
  if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc"; tail -n 40 "gpurun_out/$name.log"; exit $rc; fi
}
run j22_pipe 200 python -u -m pytest tests/test_attn_bwd_gpu.py -x -q -s -m gpu -k "pipe or split" --timeout 60 --timeout-method thread
run j22_kbwd 400 python tools/kbench.py attn_bwd
run j22_train0 400 python tools/kbench.py train
SR_ATTN_BWD_QSPLIT=1 run j22_train1 400 python tools/kbench.py train
