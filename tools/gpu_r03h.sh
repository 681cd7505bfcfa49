#!/bin/bash
# Persistent gated decode paths + RS(20,30) row-pipelined default: GPU suite, decode path A/B
# (gate vs plan path vs direct) on RS(20,30) / RS(16,24) single and multi, per-block latency.
# usage: tools/gpu_r03h.sh TAG
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
for spec in "20 10 0" "20 10 10" "16 8 8" "16 8 0"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --tiers --k $1 --m $2 --blocks 524288 --multi $3 --rounds 5 > "$O/paths_$1_$3.log" 2>&1
  tail -1 "$O/paths_$1_$3.log"
done
timeout -k 10 120 python -u tools/per_block_latency.py > "$O/per_block_latency.log" 2>&1
cat "$O/per_block_latency.log"
