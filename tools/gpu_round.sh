#!/bin/bash
# One GPU box call that refreshes every measured artifact of a round (run through gpurun from
# the repo root; each GPU step under its own time limit, steps chained so the first failure
# ends the call):
#   gpu tests -> bench.py -> rocprofv3 kernel stats of bench.py -> PMC FETCH_SIZE / WRITE_SIZE
#   passes -> per-kernel HBM bytes -> every BASELINE config (tools/config_bench.py)
# usage: tools/gpu_round.sh TAG      (outputs under gpurun_out/TAG/)
set -eo pipefail
TAG=${1:?tag}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail=3 -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
tail -2 "$O/pytest_gpu.log"
timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > "$O/smoke.log" 2>&1
tail -1 "$O/smoke.log"
timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1
tail -1 "$O/bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --no-cpu-baseline > "$O/prof.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$O/pmc_write.log" 2>&1
cd "$R"
python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_traffic.json" > /dev/null
python tools/trace_summary.py "$O/prof" "$O/kernel_trace_summary.json" > /dev/null
timeout -k 10 300 python -u tools/config_bench.py > "$O/config_bench.log" 2>&1
grep -v amdgpu.ids "$O/config_bench.log"
# host-resident Go-ABI throughput (one host thread, submit + poll), then counters for the
# configs furthest from the roofline
for c in "rs 8 4 65536 2048 1200 1" "rs 8 4 65536 2048 1200 8" "rs 20 10 32768 1024 1200 1" "rs 20 10 32768 1024 1200 8" "rs 2 1 131072 4096 1200 8" "xor 2 1 131072 4096 1200 8"; do
  for mode in copy ref; do   # ref: both sides by reference from the registered pool (RS)
    timeout -k 10 90 "$R/0xfec_amd/_bin/go_batch_bench" $c $mode
  done
done > "$O/go_batch_bench.log" 2>&1
cat "$O/go_batch_bench.log"
tools/pmc_configs.sh "$TAG/counters" "rs1624,rs2030m,rs23"
