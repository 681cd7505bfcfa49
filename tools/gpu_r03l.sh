#!/bin/bash
# Table-copy rebuild as the default (dec_fixk 4): GPU suite, bench, every config, the rebuild A/B on
# RS(16,24) / RS(20,30), and counter passes on the two multi-erasure configs.
# usage: tools/gpu_r03l.sh TAG
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --host-blocks 0 > "$O/bench.log" 2>&1
tail -1 "$O/bench.log" | cut -c1-300
timeout -k 10 300 python -u tools/config_bench.py > "$O/config_bench.log" 2>&1
grep -v amdgpu.ids "$O/config_bench.log"
for spec in "16 8 8" "20 10 10"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --k $1 --m $2 --blocks 524288 --multi $3 --rounds 7 \
    --only "fixk" > "$O/ab_$1_$3.log" 2>&1
  tail -1 "$O/ab_$1_$3.log"
done
bash tools/pmc_configs.sh "$TAG/pmc" rs1624,rs2030m
