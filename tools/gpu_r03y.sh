#!/bin/bash
# Kernel times of the sorted plan kernel and the rebuild for each plan-sort window.
set -eo pipefail
R=$(pwd)
O=$R/gpurun_out/r03y
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for spec in "16 8 8" "20 10 10"; do
  for ps in -1 1; do
    set -- $spec
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p_$1_$ps" -o run -- \
      python3 "$R/tools/plan_sort_probe.py" $1 $2 $3 $ps > "$O/p_$1_$ps.log" 2>&1
    echo "== RS($1) psort $ps"
    grep -h "plan_sorted\|rebuild_k" "$O/p_$1_$ps"/*kernel_stats.csv | cut -d, -f1-5 | cut -c1-160
  done
done
