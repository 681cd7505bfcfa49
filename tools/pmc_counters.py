#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc runs (any counters, any number of pass directories) per kernel:
the average per dispatch of each counter (summed over the XCD / shader-engine rows of one
dispatch), plus derived figures:
  valu_insts_per_wave   SQ_INSTS_VALU / SQ_WAVES
  vmem_rd_per_wave      SQ_INSTS_VMEM_RD / SQ_WAVES
  valu_active_frac      SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of a wave's life issuing VALU)
  wait_frac             SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier)
  valu_simd_util        SQ_ACTIVE_INST_VALU * 4 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
                        (quad-cycles -> cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs)
  lds_conflict_frac     SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (LDS cycles lost to bank conflicts)
  lds_busy_frac         SQ_LDS_IDX_ACTIVE / (256 CUs * GRBM_GUI_ACTIVE / 8)
  clock_ghz             GRBM_GUI_ACTIVE / 8 / kernel duration (when a kernel-trace is present)
  read_bytes / write_bytes  2 * FETCH_SIZE KiB (gfx950 correction) / WRITE_SIZE KiB

usage: pmc_counters.py OUT_JSON PASS_DIR [PASS_DIR ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirs):
    vals = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> sum
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    key = (row.get("Kernel_Name", "?"), d, row.get("Dispatch_Id"))
                    vals[key][row["Counter_Name"]] += float(row["Counter_Value"])
    per = defaultdict(lambda: defaultdict(list))
    for (name, _, _), cs in vals.items():
        for c, v in cs.items():
            per[name][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}, \
           {k: max(len(v) for v in cs.values()) for k, cs in per.items()}


def main():
    dst, dirs = sys.argv[1], sys.argv[2:]
    avg, n = load(dirs)
    res = {}
    for k in sorted(avg):
        if not k.startswith("void fk::"):
            continue
        c = dict(avg[k])
        d = {"dispatches": n[k], "counters": c}
        w = c.get("SQ_WAVES")
        if w:
            if "SQ_INSTS_VALU" in c:
                d["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / w
            if "SQ_INSTS_VMEM_RD" in c:
                d["vmem_rd_per_wave"] = c["SQ_INSTS_VMEM_RD"] / w
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            if "SQ_ACTIVE_INST_VALU" in c:
                d["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] / wc
            if "SQ_WAIT_ANY" in c:
                d["wait_frac"] = c["SQ_WAIT_ANY"] / wc
        g = c.get("GRBM_GUI_ACTIVE")
        if g and "SQ_ACTIVE_INST_VALU" in c:
            d["valu_simd_util"] = c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * g / 8)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            # share of the LDS's indexed-access cycles lost to bank conflicts
            d["lds_conflict_frac"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        if g and "SQ_LDS_IDX_ACTIVE" in c:
            # LDS busy share of the kernel's cycles, per CU (256 CUs; GRBM_GUI_ACTIVE summed over 8 XCDs)
            d["lds_busy_frac"] = c["SQ_LDS_IDX_ACTIVE"] / (256 * g / 8)
        if "FETCH_SIZE" in c:
            d["read_bytes"] = 2 * c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            d["write_bytes"] = c["WRITE_SIZE"] * 1024
        res[k] = d
    with open(dst, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
