#!/bin/bash
# The one GPU-box script (run through gpurun from the repo root). Every GPU step runs under its own
# time limit and the steps are chained (set -e), so the first failure ends the call.
#
# usage: tools/gpu_round.sh TAG [STEP ...]          outputs under gpurun_out/TAG/
# default steps (a round's refresh of every judged artifact):
#   tests smoke bench prof pmc configs go counters
# steps:
#   tests       pytest -m gpu (the whole GPU suite)
#   variants    pytest -m gpu -k kernel_variants / plan_forms (every shipped kernel path against the oracle)
#   smoke       __graft_entry__.smoke()
#   bench       bench.py (the contract line)
#   prof        rocprofv3 --kernel-trace --stats of bench.py -> kernel_trace_summary.json
#   pmc         rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py -> pmc_traffic.json
#   configs     tools/config_bench.py (every BASELINE config, device-resident)
#   go          tools/go_batch_bench (host-resident Go ABI, copy and ref submit)
#   burst       tools/go_batch_bench burst (receive-side run-loop stall per burst, p50 / p99)
#   counters    SQ / TCC / LDS counter passes of the configs furthest from the roofline
#   dectwin     tools/dec_twin_probe.py (RS(8,12) decode and its traffic twins at every residency)
#   torchrun1   bench.py under torchrun with one rank (the RCCL branch on one device)
#   rehearse2   bench.py --gpus 2 --rehearse-one-gpu (the N-rank code path, gloo, one device)
#   hostsweep   tools/host_chunk_sweep.py (host-resident pipeline chunk size)
#   hostthreads tools/host_chunk_sweep.py --threads (pageable staging copy threads)
#   twins       tools/twin_sweep.py (RS(8,12) encode and its traffic twin at several residencies)
#   duplex      tools/pcie_duplex_probe (host link per direction and both at once)
#   zerocopy    tools/zerocopy_probe (kernel reads of pinned host memory)
set -eo pipefail
TAG=${1:?tag}
shift
STEPS=${*:-tests smoke bench prof pmc configs go counters}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
PYT="python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread"

for s in $STEPS; do
  echo "== $s"
  case $s in
    tests)
      timeout -k 10 600 $PYT tests --maxfail=3 > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
      tail -2 "$O/pytest_gpu.log" ;;
    variants)
      timeout -k 10 300 $PYT tests/test_gpu_codec.py -x -k "kernel_variants or plan_forms" > "$O/pytest_variants.log" 2>&1 || { tail -30 "$O/pytest_variants.log"; exit 1; }
      tail -1 "$O/pytest_variants.log" ;;
    smoke)
      timeout -k 10 120 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$O/smoke.log" 2>&1
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$O/bench.log" 2>&1
      tail -1 "$O/bench.log" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run \
        -- python3 "$R/bench.py" --steps 20 --no-cpu-baseline > "$O/prof.log" 2>&1)
      python tools/trace_summary.py "$O/prof" "$O/kernel_trace_summary.json" > /dev/null ;;
    pmc)
      (cd /tmp && export TMPDIR=/tmp &&
       timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run \
         -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --host-blocks 0 > "$O/pmc_fetch.log" 2>&1 &&
       timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run \
         -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --host-blocks 0 > "$O/pmc_write.log" 2>&1)
      python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_traffic.json" > /dev/null ;;
    configs)
      timeout -k 10 300 python -u tools/config_bench.py > "$O/config_bench.log" 2>&1
      grep -v amdgpu.ids "$O/config_bench.log" ;;
    go)
      for c in "rs 8 4 65536 2048 1200 1" "rs 8 4 65536 2048 1200 8" "rs 20 10 32768 1024 1200 1" "rs 20 10 32768 1024 1200 8" \
               "rs 2 1 131072 4096 1200 8" "xor 2 1 131072 4096 1200 8"; do
        for mode in copy ref; do   # ref: both sides by reference from the registered pool (RS)
          timeout -k 10 90 "$R/0xfec_amd/_bin/go_batch_bench" $c $mode
        done
      done > "$O/go_batch_bench.log" 2>&1
      cat "$O/go_batch_bench.log" ;;
    burst)
      for km in "8 4" "20 10"; do
        for n in 1 8 64; do
          for mode in copy ref; do
            for zc in 0 4194304; do   # the decoder's zero-copy sets (knob bat_zc) off / up to 4 MiB
              timeout -k 10 90 "$R/0xfec_amd/_bin/go_batch_bench" burst $km $n 400 1200 $mode zc=$zc
            done
          done
        done
      done > "$O/go_burst.log" 2>&1
      cat "$O/go_burst.log" ;;
    counters)
      tools/pmc_configs.sh "$TAG/counters" "rs1624,rs2030m,rs23" ;;
    dectwin)
      timeout -k 10 400 python -u tools/dec_twin_probe.py > "$O/dec_twin.log" 2>&1
      grep -v amdgpu.ids "$O/dec_twin.log" | tail -60 ;;
    torchrun1)
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29611 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --host-blocks 0 > "$O/bench_torchrun_n1_rccl.log" 2>&1
      tail -1 "$O/bench_torchrun_n1_rccl.log" | cut -c1-400 ;;
    rehearse2)
      timeout -k 10 300 python bench.py --gpus 2 --rehearse-one-gpu --steps 10 --warmup 3 --no-cpu-baseline --host-blocks 0 \
        > "$O/bench_n2_rehearse.log" 2>&1
      tail -1 "$O/bench_n2_rehearse.log" | cut -c1-400 ;;
    twins)
      timeout -k 10 300 python -u tools/twin_sweep.py > "$O/twin_sweep.log" 2>&1
      grep -v amdgpu.ids "$O/twin_sweep.log" ;;
    hostsweep)
      timeout -k 10 400 python -u tools/host_chunk_sweep.py --chunks 0,3072,4096,6144,8192 > "$O/host_chunk_sweep.log" 2>&1
      grep -v amdgpu.ids "$O/host_chunk_sweep.log" | cut -c1-400 ;;
    hostthreads)
      timeout -k 10 400 python -u tools/host_chunk_sweep.py --threads 8,12,16 --reps 3 > "$O/host_thread_sweep.log" 2>&1
      grep -v amdgpu.ids "$O/host_thread_sweep.log" | tail -1 ;;
    duplex)
      timeout -k 10 120 tools/pcie_duplex_probe > "$O/pcie_duplex_probe.log" 2>&1
      cat "$O/pcie_duplex_probe.log" ;;
    zerocopy)
      timeout -k 10 120 tools/zerocopy_probe 131072 4 > "$O/zerocopy_probe.log" 2>&1
      cat "$O/zerocopy_probe.log" ;;
    *)
      echo "unknown step $s" >&2; exit 2 ;;
  esac
done
