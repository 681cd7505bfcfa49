#!/bin/bash
# Zero-copy host-read probe, then the decode path A/B (two-tier rebuild, big-code direct kernel,
# device-side gate) on the reference's RS(20,30) and BASELINE config #4 RS(16,24).
# usage: tools/gpu_r03d.sh TAG   (outputs under gpurun_out/TAG/)
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 120 tools/zerocopy_probe 131072 4 > "$O/zerocopy_probe.log" 2>&1
cat "$O/zerocopy_probe.log"
timeout -k 10 120 tools/zerocopy_probe 32768 4 > "$O/zerocopy_probe_32k.log" 2>&1
cat "$O/zerocopy_probe_32k.log"
for spec in "20 10 0" "20 10 10" "16 8 8" "16 8 0"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --tiers --k $1 --m $2 --blocks 524288 --multi $3 --rounds 5 > "$O/paths_$1_$3.log" 2>&1
  tail -1 "$O/paths_$1_$3.log"
done
