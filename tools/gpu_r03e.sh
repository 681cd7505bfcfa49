#!/bin/bash
# Go-ABI by-reference submit (registered pool + device gather) and the pinned decode's parity
# gather: their GPU tests, then the Go-ABI bench copy vs ref, then bench.py's host_resident leg.
# usage: tools/gpu_r03e.sh TAG   (outputs under gpurun_out/TAG/)
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_go_ref.py tests/test_go_harness.py tests/test_gpu_batch.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_ref.log" 2>&1 || { tail -30 "$O/pytest_ref.log"; exit 1; }
tail -2 "$O/pytest_ref.log"
for c in "rs 8 4 65536 2048 1200 1" "rs 8 4 65536 2048 1200 1 ref" "rs 8 4 65536 2048 1200 8" "rs 8 4 65536 2048 1200 8 ref" "rs 20 10 32768 1024 1200 1" "rs 20 10 32768 1024 1200 1 ref" "rs 20 10 32768 1024 1200 8 ref"; do
    timeout -k 10 90 0xfec_amd/_bin/go_batch_bench $c
done > "$O/go_batch_bench.log" 2>&1
cat "$O/go_batch_bench.log"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$O/bench.log" 2>&1
tail -1 "$O/bench.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], json.dumps(d['host_resident']))"
