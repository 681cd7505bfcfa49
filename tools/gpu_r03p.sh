#!/bin/bash
# The bench's torchrun branch on real RCCL with one rank (init_process_group("nccl"), barriers,
# all_gather / all_reduce of the step times and checks), then the 2-rank gloo rehearsal.
set -eo pipefail
O=gpurun_out/r03p
mkdir -p "$O"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --host-blocks 0 > "$O/bench_torchrun_n1_rccl.log" 2>&1
tail -1 "$O/bench_torchrun_n1_rccl.log" | cut -c1-400
timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline --host-blocks 0 > "$O/bench_n2_rehearse.log" 2>&1
tail -1 "$O/bench_n2_rehearse.log" | cut -c1-400
