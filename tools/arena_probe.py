#!/usr/bin/env python3
"""Diagnostics: RS(8,12) encode and single-erasure decode (bench.py's workload, 2^20 blocks) on
two buffer arrangements in one process, timed alternately: "separate" (bench.py's RankBatch: data,
parity and recovered as separate torch allocations) and "arena" (the same three regions carved
back to back out of one allocation). Says whether bench.py's own allocation pattern costs rate
against one contiguous allocation.

usage: arena_probe.py [blocks] [rounds] [--more (three more arrangements)] [--sweep (the gap between
       data and parity in one allocation)] [--order (which region lies above which)]
       [--arena-first] [--interleaved | --interleaved-first (each block's n
       shards contiguous)]"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402  (padded)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 1 << 20
    rounds = int(args[1]) if len(args) > 1 else 6
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, L, S = 8, 4, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    codec.prepare(k, m)
    nd, npar, no = B * k * S, B * m * S, B * S
    masks = torch.empty((B,), dtype=torch.int32, device="cuda")
    codec.synth_single_erasures(0x0FEC, 0, B, k, m, masks.data_ptr(), None)
    lay, keep = {}, []

    def separate():
        data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
        par = bench.padded(torch, (B, m, S), "cuda")
        rec = bench.padded(torch, (B, 1, S), "cuda")
        keep.extend((data, par, rec))
        lay["separate"] = (data.data_ptr(), par.data_ptr(), rec.data_ptr())

    def arena():
        a = torch.zeros(nd + npar + no, dtype=torch.uint8, device="cuda")
        keep.append(a)
        a0 = a.data_ptr()
        lay["arena"] = (a0, a0 + nd, a0 + nd + npar)
    def interleaved():
        # each block's k data and m parity shards contiguous ([B][n][S], the batch layer's staging
        # layout), the recovered shards after them
        il = torch.zeros(B * (k + m) * S + no, dtype=torch.uint8, device="cuda")
        keep.append(il)
        i0 = il.data_ptr()
        lay["interleaved"] = (i0, i0 + k * S, i0 + B * (k + m) * S)
    # --arena-first: the arena is allocated before the separate buffers (the first allocations of
    # a process take the first device memory the runtime hands out); --interleaved: the
    # interleaved layout too, allocated last, or first with --interleaved-first
    order = [arena, separate] if "--arena-first" in sys.argv else [separate, arena]
    if "--interleaved-first" in sys.argv:
        order = [interleaved] + order
    elif "--interleaved" in sys.argv:
        order = order + [interleaved]
    for f in order:
        f()
    if "--more" in sys.argv:
        # regions in the other order; with 1 GiB gaps between them; data alone + parity and
        # recovered in a second allocation
        rev = torch.zeros(nd + npar + no, dtype=torch.uint8, device="cuda")
        r0 = rev.data_ptr()
        lay["arena_rev"] = (r0 + npar, r0, r0 + npar + nd)
        G = 1 << 30
        gap = torch.zeros(nd + npar + no + 2 * G, dtype=torch.uint8, device="cuda")
        g0 = gap.data_ptr()
        lay["arena_gap1G"] = (g0, g0 + nd + G, g0 + nd + npar + 2 * G)
        d2 = torch.empty(nd, dtype=torch.uint8, device="cuda")
        po = torch.zeros(npar + no, dtype=torch.uint8, device="cuda")
        lay["two_allocs"] = (d2.data_ptr(), po.data_ptr(), po.data_ptr() + npar)
    if "--order" in sys.argv:
        # which region sits above which: separate allocations made in the reverse order (the
        # runtime hands out decreasing addresses, so data ends up lowest), and one-allocation
        # orders with parity below data
        rec2 = bench.padded(torch, (B, 1, S), "cuda")
        par2 = bench.padded(torch, (B, m, S), "cuda")
        data2 = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
        lay["separate_rev"] = (data2.data_ptr(), par2.data_ptr(), rec2.data_ptr())
        G = 1 << 30
        o = torch.zeros(nd + npar + no + G, dtype=torch.uint8, device="cuda")
        o0 = o.data_ptr()
        lay["par_gap_data_rec"] = (o0 + npar + G, o0, o0 + npar + G + nd)
        o2 = torch.zeros(nd + npar + no, dtype=torch.uint8, device="cuda")
        q0 = o2.data_ptr()
        lay["data_rec_par"] = (q0, q0 + nd + no, q0 + nd)
        lay["rec_data_par"] = (q0 + no, q0 + no + nd, q0)
    if "--sweep" in sys.argv:
        # parity placed `gap` bytes after the end of data in one allocation, recovered right
        # after parity (a rank's batch as one arena, the gap swept)
        MB = 1 << 20
        gaps = [0, 2 * MB, 16 * MB, 64 * MB, 256 * MB, 512 * MB, 768 * MB, 1024 * MB, 1536 * MB,
                2048 * MB, 3072 * MB, 4096 * MB]
        big = torch.zeros(nd + npar + no + gaps[-1], dtype=torch.uint8, device="cuda")
        b0 = big.data_ptr()
        for g in gaps:
            lay["gap%dM" % (g // MB)] = (b0, b0 + nd + g, b0 + nd + g + npar)
        del lay["separate"], lay["arena"]
    strides = {nm: ((k + m) * S, (k + m) * S) if nm == "interleaved" else (k * S, m * S) for nm in lay}
    for nm, (dp, _, _) in lay.items():
        codec.synth_data(0x0FEC, 0, B, k, 1200, dp, strides[nm][0], S)

    def timed(fn, n=20):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n

    res = {}
    for _ in range(rounds):
        for name, (dp, pp, op) in lay.items():
            dbs, pbs = strides[name]

            def enc():
                codec.rs_encode_raw(k, m, L, B, dp, dbs, pp, pbs, S, fec.FEC_DEVICE)

            def dec():
                rc = codec.rs_recover_raw(k, m, L, B, dp, dbs, pp, pbs, S, masks.data_ptr(), op, S, 1, None)
                assert rc == 0
            res.setdefault(name + " encode", []).append(timed(enc))
            res.setdefault(name + " decode", []).append(timed(dec))
    med = {n: round(sorted(v)[len(v) // 2], 4) for n, v in res.items()}
    addrs = {n: [hex(x) for x in v] for n, v in lay.items()}
    print(json.dumps({"blocks": B, "median_ms": med, "addresses": addrs}), flush=True)


if __name__ == "__main__":
    main()
