#!/bin/bash
# Round-3 refresh after the RS(20,30) row-pipelined rebuild became the default: the GPU suite,
# every config, counters of the multi-erasure rebuilds, per-block latency of the per-block schemes.
# usage: tools/gpu_r03g.sh TAG
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -u tools/config_bench.py > "$O/config_bench.log" 2>&1
grep -v amdgpu.ids "$O/config_bench.log"
timeout -k 10 120 python -u tools/per_block_latency.py > "$O/per_block_latency.log" 2>&1
cat "$O/per_block_latency.log"
tools/pmc_configs.sh "$TAG/counters" "rs2030m,rs1624"
