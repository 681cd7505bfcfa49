#!/bin/bash
# Round-3 first GPU call on the restored tree: the stream-switch probe, then tools/gpu_round.sh
# (suite, smoke, bench, rocprof stats, PMC traffic, every config, Go-ABI rates, counters), then
# the N>1 launcher rehearsal and the N=8 refusal. Outputs under gpurun_out/TAG/.
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 120 python -u tools/stream_switch_probe.py > "$O/stream_probe.log" 2>&1
tail -1 "$O/stream_probe.log"
tools/gpu_round.sh "$TAG"
timeout -k 10 200 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline --host-blocks 0 > "$O/bench_n2_rehearse.log" 2>&1
tail -1 "$O/bench_n2_rehearse.log"
set +e
timeout -k 10 120 python -u bench.py --gpus 8 > "$O/bench_n8_refused.log" 2>&1
echo "bench --gpus 8 on one GPU: rc=$?"
tail -2 "$O/bench_n8_refused.log"
