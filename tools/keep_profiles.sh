#!/bin/bash
# Copy the judged artifacts of one tools/gpu_round.sh call (gpurun_out/TAG) into profiles/rNN/
# with the tag in their names, and point bench.py's PMC traffic at that call's profile.
# usage: tools/keep_profiles.sh TAG ROUND_DIR     e.g. tools/keep_profiles.sh r03b r03
set -eo pipefail
TAG=${1:?tag}; RD=${2:?round dir}
S=gpurun_out/$TAG
D=profiles/$RD
mkdir -p "$D"
cp_if() { [ -f "$1" ] && cp "$1" "$2" || true; }
cp_if "$S/bench.log" "$D/bench_$TAG.log"
cp_if "$S/smoke.log" "$D/smoke_$TAG.log"
cp_if "$S/pytest_gpu.log" "$D/pytest_gpu_$TAG.log"
cp_if "$S/config_bench.log" "$D/config_bench_$TAG.log"
cp_if "$S/go_batch_bench.log" "$D/go_batch_bench_$TAG.log"
cp_if "$S/stream_probe.log" "$D/stream_probe_$TAG.log"
cp_if "$S/bench_n2_rehearse.log" "$D/bench_n2_rehearse_$TAG.log"
cp_if "$S/bench_n8_refused.log" "$D/bench_n8_refused_$TAG.log"
cp_if "$S/kernel_trace_summary.json" "$D/bench_${TAG}_kernel_trace_summary.json"
cp_if "$S/prof/run_kernel_stats.csv" "$D/bench_${TAG}_kernel_stats.csv"
cp_if "$S/pmc_traffic.json" "$D/pmc_traffic_$TAG.json"
cp_if "$S/counters/counters.json" "$D/counters_$TAG.json"
cp_if "$S/go_burst.log" "$D/go_burst_$TAG.log"
cp_if "$S/pcie_duplex_probe.log" "$D/pcie_duplex_probe_$TAG.log"
cp_if "$S/zerocopy_probe.log" "$D/zerocopy_probe_$TAG.log"
cp_if "$S/pytest_variants.log" "$D/pytest_variants_$TAG.log"
cp_if "$S/host_chunk_sweep.log" "$D/host_chunk_sweep_$TAG.log"
cp_if "$S/host_thread_sweep.log" "$D/host_thread_sweep_$TAG.log"
cp_if "$S/twin_sweep.log" "$D/twin_sweep_$TAG.log"
cp_if "$S/bench_torchrun_n1_rccl.log" "$D/bench_torchrun_n1_rccl_$TAG.log"
for f in "$S"/ab_*.log "$S"/enc_*.log; do cp_if "$f" "$D/$(basename "$f" .log)_$TAG.log"; done
for d in "$S"/counters_*/; do cp_if "$d/counters.json" "$D/$(basename "$d")_$TAG.json"; done
if [ -f "$S/pmc_traffic.json" ]; then cp "$S/pmc_traffic.json" profiles/pmc_traffic_latest.json; fi
ls "$D" | grep "$TAG"
