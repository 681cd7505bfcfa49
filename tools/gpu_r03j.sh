#!/bin/bash
# Table-copy rebuild (fec_rebuild.hip, dec_fixk 4): parity of the variant against the oracle, then an
# interleaved A/B against the default rebuild on RS(16,24) and RS(20,30) multi-erasure batches.
# usage: tools/gpu_r03j.sh TAG
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "kernel_variants and (16-8 or 20-10)" > "$O/pytest_variants.log" 2>&1 || { tail -30 "$O/pytest_variants.log"; exit 1; }
tail -2 "$O/pytest_variants.log"
for spec in "16 8 8" "20 10 10"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --k $1 --m $2 --blocks 524288 --multi $3 --rounds 7 \
    --only "fixk 4" > "$O/ab_$1_$3.log" 2>&1
  tail -1 "$O/ab_$1_$3.log"
done
