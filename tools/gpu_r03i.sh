#!/bin/bash
# After reverting the persistent wave-rebuild loop: GPU suite, bench, decode path A/B on
# RS(20,30) / RS(16,24), every config. usage: tools/gpu_r03i.sh TAG
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --host-blocks 0 > "$O/bench.log" 2>&1
tail -1 "$O/bench.log" | cut -c1-300
for spec in "20 10 0" "20 10 10" "16 8 8"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --tiers --k $1 --m $2 --blocks 524288 --multi $3 --rounds 5 > "$O/paths_$1_$3.log" 2>&1
  tail -1 "$O/paths_$1_$3.log"
done
timeout -k 10 300 python -u tools/config_bench.py > "$O/config_bench.log" 2>&1
grep -v amdgpu.ids "$O/config_bench.log"
