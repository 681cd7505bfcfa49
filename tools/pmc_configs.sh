#!/bin/bash
# Counter passes over tools/config_bench.py configs (one rocprofv3 run per pass, each under its
# own time limit; chained so the first failure ends the call):
#   pass A  SQ: waves, VALU / VMEM instructions, wave cycles, VALU-active, waits, busy + GRBM clock
#   pass B  TCC FETCH_SIZE            pass C  TCC WRITE_SIZE
#   pass D  LDS: instructions, index-active and bank-conflict cycles, LDS issue / wait cycles
# usage (from the repo root, on the GPU box): tools/pmc_configs.sh TAG CONFIG[,CONFIG..] [config_bench args]
set -eo pipefail
TAG=${1:?tag}; ONLY=${2:?configs}; shift 2
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $A --output-format csv -d "$O/pmc_sq" -o run -- python3 "$R/tools/config_bench.py" --only "$ONLY" --iters 5 "$@" > "$O/pmc_sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python3 "$R/tools/config_bench.py" --only "$ONLY" --iters 5 "$@" > "$O/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- python3 "$R/tools/config_bench.py" --only "$ONLY" --iters 5 "$@" > "$O/pmc_write.log" 2>&1
D="SQ_WAVES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $D --output-format csv -d "$O/pmc_lds" -o run -- python3 "$R/tools/config_bench.py" --only "$ONLY" --iters 5 "$@" > "$O/pmc_lds.log" 2>&1
cd "$R"
python3 tools/pmc_counters.py "$O/counters.json" "$O/pmc_sq" "$O/pmc_fetch" "$O/pmc_write" "$O/pmc_lds" > /dev/null
python3 - "$O/counters.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    print(k[:70], {x: round(y, 3) for x, y in v.items() if not isinstance(y, dict) and x != "dispatches"})
PY
