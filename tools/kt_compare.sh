#!/bin/bash
# kernel traces of dec_select (RS(16,24) multi) and config_bench rs1624, for comparing the launches
set -eo pipefail
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_sel" -o run -- python3 "$R/tools/dec_select.py" --k 16 --m 8 --blocks 524288 --multi 8 --rounds 1 --iters 3 > "$R/gpurun_out/kt_sel.log" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_cb" -o run -- python3 "$R/tools/config_bench.py" --only rs1624 --iters 3 > "$R/gpurun_out/kt_cb.log" 2>&1
