#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace run, split by launch size (grid), so the
full-size launches of bench.py's timed steps are not averaged with the same kernels' small
launches from its checks and host-resident leg.

usage: trace_summary.py PROF_DIR [OUT_JSON]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if not name.startswith("void fk::"):
            continue
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        by[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {}
    for (name, grid), v in sorted(by.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        v.sort()
        out.setdefault(name, []).append({"grid_threads": grid, "calls": len(v), "avg_ms": round(sum(v) / len(v) / 1e6, 4),
                                         "median_ms": round(v[len(v) // 2] / 1e6, 4), "min_ms": round(v[0] / 1e6, 4),
                                         "max_ms": round(v[-1] / 1e6, 4)})
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main()
