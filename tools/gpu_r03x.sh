#!/bin/bash
# Plan records sorted over 128-block windows (dec_psort): parity of every variant, then the A/B.
set -eo pipefail
O=gpurun_out/r03x
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "kernel_variants" > "$O/pytest_variants.log" 2>&1 || { tail -30 "$O/pytest_variants.log"; exit 1; }
tail -1 "$O/pytest_variants.log"
for spec in "16 8 8" "20 10 10"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --k $1 --m $2 --blocks 524288 --multi $3 --rounds 7 \
    --only "blocks" > "$O/ab_$1_$3.log" 2>&1
  tail -1 "$O/ab_$1_$3.log"
done
bash tools/gpu_r03y.sh
