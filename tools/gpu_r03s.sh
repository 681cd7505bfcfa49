#!/bin/bash
# Table-copy rebuild residency caps (dec_wpc 2, 3 against the uncapped 4 workgroups/CU).
set -eo pipefail
O=gpurun_out/r03s
mkdir -p "$O"
for spec in "16 8 8" "20 10 10"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --k $1 --m $2 --blocks 524288 --multi $3 --rounds 7 \
    --only "fixk 4) wpc" > "$O/ab_$1_$3.log" 2>&1
  tail -1 "$O/ab_$1_$3.log"
done
