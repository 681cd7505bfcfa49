set -eo pipefail
R=$(pwd)
timeout -k 10 120 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread -k "recover" > gpurun_out/rs23_t.log 2>&1
timeout -k 10 120 python -u tools/dec_select.py --k 2 --m 1 --blocks 65536 --rounds 6 --iters 50 > gpurun_out/rs23_sel.log 2>&1
timeout -k 10 120 python -u tools/config_bench.py --only rs23,rs812 > gpurun_out/rs23_cb.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/rs23_prof" -o run -- python3 "$R/tools/config_bench.py" --only rs23 > "$R/gpurun_out/rs23_prof.log" 2>&1
