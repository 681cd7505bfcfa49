#!/usr/bin/env python3
"""Static VALU split of the multi-erasure rebuild (fec_rebuild.hip rs_rebuild_k_kernel) by work
category, per row-count body, and the expected VALU per wave for a loss distribution (round 6,
VERDICT r5 item 3: where RS(20,30)'s ~2000 VALU per wave go before choosing a cut).

The kernel's device assembly (hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S) is cut at the
`; rows N` markers the row bodies open with (fec_rebuild.hip rebuild_rows); the code before the
first marker is the wave's prologue (table copy, plan records, PermTab rows, input offsets: run
once per wave whatever its row count). Categories, by opcode:
  products  v_perm_b32 (3 per coefficient and dword)
  folds     v_bitop3_b32 / v_xor_b32 (three-input XORs folding products into the accumulators)
  splits    v_and_b32 / v_lshrrev_b32 / v_bfe_u32 / v_and_or_b32 / v_lshrrev_b64 (x & 7, x >> 3 & 7,
            x >> 6 & 3 per input dword)
  address   v_add* / v_lshl* / v_mad* / v_mov_b64 / v_readfirstlane (load and store addresses)
  other     the rest (selects, compares, moves)
Expected VALU per wave = prologue + sum over r of P(wave rows = r) * body_r, with the wave's row
count taken as the erased data shards of its block (sorted plans: a wave's blocks have nearly
always the same count) under e ~ U{1..MULTI} losses spread uniformly over the n shards.

usage: valu_split.py FILE.s K M MULTI"""
import sys
from collections import Counter
from fractions import Fraction
from math import comb

CATS = (("products", ("v_perm_b32",)),
        ("folds", ("v_bitop3_b32", "v_xor_b32")),
        ("splits", ("v_and_b32", "v_lshrrev_b32", "v_bfe_u32", "v_and_or_b32", "v_lshrrev_b64")),
        ("address", ("v_add", "v_lshl", "v_mad", "v_mov_b64", "v_readfirstlane", "v_sub", "v_mul")))


def cat(op):
    for name, pre in CATS:
        if any(op.startswith(p) for p in pre):
            return name
    return "other"


def split_kernel(lines, k, m):
    sym = "rs_rebuild_k_kernelILi%dELi%dE" % (k, m)
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    parts, cur = {}, "prologue"
    for l in lines[start:end]:
        t = l.strip()
        if t.startswith("; rows "):
            cur = int(t.split()[2])
            continue
        if not l.startswith("\t") or t.startswith((".", ";")) or not t:
            continue
        op = t.split()[0]
        parts.setdefault(cur, Counter())[cat(op) if op.startswith("v_") else ("stores" if op.startswith("global_store") else ("loads" if op.startswith("global_load") else "nonvalu"))] += 1
    return parts


def rows_dist(k, m, multi):
    n = k + m
    p = Counter()
    for e in range(1, multi + 1):
        for d in range(0, min(e, k) + 1):
            p[d] += Fraction(1, multi) * Fraction(comb(k, d) * comb(m, e - d), comb(n, e))
    return p


def main():
    path, k, m, multi = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    parts = split_kernel(open(path).read().split("\n"), k, m)
    keys = ("products", "folds", "splits", "address", "other")
    print("body       " + " ".join("%9s" % c for c in keys) + "     VALU  loads stores")
    for b in ["prologue"] + sorted(x for x in parts if x != "prologue"):
        c = parts[b]
        print("%-10s " % b + " ".join("%9d" % c[x] for x in keys) + " %8d %6d %6d" % (
            sum(c[x] for x in keys), c["loads"], c["stores"]))
    dist = rows_dist(k, m, multi)
    p0 = dist[0]
    exp = Counter()
    for r, pr in dist.items():
        if r == 0:
            continue
        for x in keys:
            exp[x] += float(pr / (1 - p0)) * parts[r][x]
    pro = parts["prologue"]
    tot = sum(exp.values()) + sum(pro[x] for x in keys)
    print("rows distribution (waves with rows > 0):", {r: round(float(v / (1 - p0)), 4) for r, v in sorted(dist.items()) if r})
    print("expected VALU per rebuilding wave: %.0f = prologue %d + bodies %.0f" % (tot, sum(pro[x] for x in keys), sum(exp.values())))
    print("  by category (prologue included): " + ", ".join("%s %.0f (%.0f %%)" % (
        x, exp[x] + pro[x], 100 * (exp[x] + pro[x]) / tot) for x in keys))


if __name__ == "__main__":
    main()
