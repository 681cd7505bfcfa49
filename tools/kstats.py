#!/usr/bin/env python3
"""Instruction mix and register use of kernels in a device assembly file
(hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S -o x.s file.hip).

usage: kstats.py FILE.s [NAME_SUBSTRING] [--top N]"""
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 0
    s = open(path).read().split("\n")
    for i, l in enumerate(s):
        if not l.startswith("_Z") or ":" not in l or pat not in l.split(":")[0]:
            continue
        name = l.split(":")[0]
        j = i
        while j < len(s) and not s[j].startswith(".Lfunc_end"):
            j += 1
        body = [x.split()[0] for x in s[i:j] if x.startswith("\t") and not x.startswith("\t.") and not x.startswith("\t;")]
        c = Counter(body)
        meta = {}
        for x in s[j:j + 80]:
            for key in (".num_vgpr,", ".numbered_sgpr,", ".private_seg_size,"):
                if name + key in x.replace(" ", ""):
                    meta[key.strip(".,")] = x.split(",")[-1].strip()
            if x.startswith("; Occupancy:") and "occ" not in meta:
                meta["occ"] = x.split(":")[1].strip()
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        print("%-70s instr %5d valu %5d vmem_ld %3d %s" % (name[:70], len(body), valu,
              sum(v for k, v in c.items() if k.startswith("global_load")), meta))
        if top:
            print("   ", c.most_common(top))


if __name__ == "__main__":
    main()
