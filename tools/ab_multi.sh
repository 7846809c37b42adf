# Interleaved kbench attn rounds: the shipped library and each tuning variant in $VLIBS.
set -o pipefail
for i in 1 2; do
  echo "== shipped"; SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py attn 2>/dev/null | grep attn || exit 1
  for v in $VLIBS; do
    echo "== $v"; SFM_AMD_LIB=$v SR_KB_STATIC=1 timeout -k 10 200 python tools/kbench.py attn 2>/dev/null | grep attn || exit 1
  done
done
