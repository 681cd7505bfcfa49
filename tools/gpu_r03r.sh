#!/bin/bash
# Sustained vs short-burst encode/decode rates (DVFS check): config_bench at 3, 20 and 60 launches
# per burst for RS(8,12) and RS(16,24), then enc_select's short interleaved bursts for RS(8,12).
set -eo pipefail
O=gpurun_out/r03r
mkdir -p "$O"
for it in 3 20 60; do
  timeout -k 10 200 python -u tools/config_bench.py --only rs812,rs1624 --iters $it > "$O/cb_iters$it.log" 2>&1
  echo "iters $it"; grep -v amdgpu.ids "$O/cb_iters$it.log" | cut -c1-220
done
timeout -k 10 300 python -u tools/enc_select.py 8,4 > "$O/enc_select_8.log" 2>&1
grep -v amdgpu.ids "$O/enc_select_8.log" | tr -d '\n ' | cut -c1-900; echo
