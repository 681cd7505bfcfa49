#!/bin/bash
# Row-pipelined rebuild (dec_fixk 3) parity + A/B, the ref-submit bench with the lock-free pool
# lookup. usage: tools/gpu_r03f.sh TAG
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -k "variants_match_oracle" tests/test_gpu_go_ref.py -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for spec in "20 10 10" "16 8 8"; do
  set -- $spec
  timeout -k 10 200 python -u tools/dec_select.py --k $1 --m $2 --blocks 524288 --multi $3 --rounds 5 > "$O/multi_$1.log" 2>&1
  tail -1 "$O/multi_$1.log"
done
for c in "rs 8 4 65536 2048 1200 1 ref" "rs 8 4 65536 2048 1200 8" "rs 8 4 65536 2048 1200 8 ref" "rs 20 10 32768 1024 1200 8 ref"; do
    timeout -k 10 90 0xfec_amd/_bin/go_batch_bench $c
done > "$O/go_batch_bench.log" 2>&1
cat "$O/go_batch_bench.log"
