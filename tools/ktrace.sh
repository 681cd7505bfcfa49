#!/bin/bash
# Kernel-trace stats of one command (rocprofv3 --kernel-trace --stats), summarised per kernel.
# usage (repo root, on the GPU box): tools/ktrace.sh TAG -- python3 tools/config_bench.py --only rs1624
set -eo pipefail
TAG=${1:?tag}; shift; [ "$1" = "--" ] && shift
R=$(pwd); O=$R/gpurun_out/$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- "$@" > "$O/kt.log" 2>&1
cd "$R"
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print("%-80s calls %5s avg_us %9.1f total_ms %8.2f" % (r["Name"][:80], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
