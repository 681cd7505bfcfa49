#!/bin/bash
# stream-switch diagnostics, then the GPU suite without that test, then the gated-path A/B
set -eo pipefail
O=gpurun_out/r03c2
mkdir -p "$O"
timeout -k 10 120 python -u tools/stream_switch_probe.py > "$O/stream_probe.log" 2>&1
tail -1 "$O/stream_probe.log"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --deselect tests/test_gpu_codec.py::test_stream_switch_orders_shared_workspace > "$O/pytest_gpu.log" 2>&1 || { grep -E "FAILED|Error|passed|failed" "$O/pytest_gpu.log" | tail -20; exit 1; }
tail -1 "$O/pytest_gpu.log"
for spec in "20 10 0" "20 10 10" "16 8 8" "16 8 0"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --tiers --k $1 --m $2 --blocks 524288 --multi $3 --rounds 5 > "$O/paths_$1_$3.log" 2>&1
  tail -1 "$O/paths_$1_$3.log"
done
