#!/bin/bash
# Decoder by-reference submit (fec_go_decoder_submit_ref): oracle tests, the Go-call harness in
# batchref mode, then the Go-ABI bench copy vs ref on one and eight host threads.
set -eo pipefail
O=gpurun_out/r03u
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_go_ref.py tests/test_go_harness.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > "$O/pytest_ref.log" 2>&1 || { tail -40 "$O/pytest_ref.log"; exit 1; }
tail -1 "$O/pytest_ref.log"
for c in "rs 8 4 65536 2048 1200 1" "rs 8 4 65536 2048 1200 8" "rs 20 10 32768 1024 1200 1" "rs 20 10 32768 1024 1200 8"; do
  for mode in copy ref; do
    timeout -k 10 90 ./0xfec_amd/_bin/go_batch_bench $c $mode
  done
done > "$O/go_batch_bench.log" 2>&1
cat "$O/go_batch_bench.log"
