#!/bin/bash
# Round-3 GPU call: the GPU suite, the bench, then the two-tier rebuild A/B (dec_select --tiers)
# on the reference's RS(20,30) (single and U{1..10} erasures) and BASELINE config #4 RS(16,24).
# usage: tools/gpu_r03_tiers.sh TAG   (outputs under gpurun_out/TAG/)
set -eo pipefail
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1
tail -1 "$O/bench.log"
timeout -k 10 200 python -u tools/dec_select.py --tiers --k 20 --m 10 --blocks 524288 --rounds 5 > "$O/tiers_2030_single.log" 2>&1
tail -1 "$O/tiers_2030_single.log"
timeout -k 10 200 python -u tools/dec_select.py --tiers --k 20 --m 10 --blocks 524288 --multi 10 --rounds 5 > "$O/tiers_2030_multi.log" 2>&1
tail -1 "$O/tiers_2030_multi.log"
timeout -k 10 200 python -u tools/dec_select.py --tiers --k 16 --m 8 --blocks 524288 --multi 8 --rounds 5 > "$O/tiers_1624_multi.log" 2>&1
tail -1 "$O/tiers_1624_multi.log"
timeout -k 10 200 python -u tools/dec_select.py --tiers --k 16 --m 8 --blocks 524288 --rounds 5 > "$O/tiers_1624_single.log" 2>&1
tail -1 "$O/tiers_1624_single.log"
timeout -k 10 200 python -u bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline --host-blocks 0 > "$O/bench_n2_rehearse.log" 2>&1
tail -1 "$O/bench_n2_rehearse.log"
set +e
timeout -k 10 120 python -u bench.py --gpus 8 > "$O/bench_n8_refused.log" 2>&1
echo "bench --gpus 8 on one GPU: rc=$?"
tail -2 "$O/bench_n8_refused.log"
