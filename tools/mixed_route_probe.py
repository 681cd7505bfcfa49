#!/usr/bin/env python3
"""Diagnostics: RS decode routes on mixed-erasure batches of the small codes (k*m*k PermTabs <=
16 KiB, the direct kernel's). Each code runs a batch with e ~ U{1..MULTI} losses uniform over all
n shards (every block recoverable), m output slots per block (a caller that does not scan the
masks first), through the default route, the sorted-plan wave route (knob dec_direct=0) and the
tile route (dec_direct=0, dec_wave=0), interleaved in one process; the outputs of the routes are
compared byte for byte. (Round 5 measured with it the direct kernel + multi-erasure worklist that
multi-slot calls took before: profiles/r05/mixed_route*_r05g.log.)

--inplace times fec_rs_reconstruct_batch (in place) instead, whose default route for RS(8,12) is the
routed one since round 6 (a classify pass, then the direct body or the sorted plans + wave rebuild
in one kernel; route "noroute" is round 5's sorted-plan route for every batch). MULTI 0: one random
data shard lost per block (bench.py's erasures).

usage: mixed_route_probe.py [blocks] [rounds] [--code K,M,MULTI ...] [--routes default,wave] [--inplace]"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

L, S = 1202, 1216
ROUTES = {"default": {}, "wave": {"dec_direct": 0}, "tile": {"dec_direct": 0, "dec_wave": 0},
          "noroute": {"dec_route": 0}, "direct_oop": {}, "route_wpc3": {"route_wpc": 3},
          "route_wpc4": {"route_wpc": 4}, "route_wpc5": {"route_wpc": 5}, "route_wpc0": {"route_wpc": 0},
          "route_ww3": {"route_ww": 3}, "route_ww3_wpc5": {"route_ww": 3, "route_wpc": 5},
          "route_ww4": {"route_ww": 4}}


def main():
    argv = sys.argv[1:]
    codes, routes = [], list(ROUTES)
    while "--code" in argv:
        i = argv.index("--code")
        codes.append(tuple(int(x) for x in argv[i + 1].split(",")))
        del argv[i:i + 2]
    if "--routes" in argv:
        i = argv.index("--routes")
        routes = argv[i + 1].split(",")
        del argv[i:i + 2]
    inplace = "--inplace" in argv
    args = [a for a in argv if not a.startswith("--")]
    B = int(args[0]) if args else 1 << 18
    rounds = int(args[1]) if len(args) > 1 else 5
    import torch
    fec = importlib.import_module("0xfec_amd")
    codec = fec.Codec(0).use_torch_stream()
    res = {}
    for k, m, multi in codes or ((8, 4, 4), (8, 4, 2), (8, 4, 1), (10, 4, 4), (4, 2, 2), (2, 2, 2)):
        n = k + m
        codec.prepare(k, m)
        g = torch.Generator(device="cuda")
        g.manual_seed(0x0FEC + k)
        data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda", generator=g)
        par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
        codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
        if multi:
            e = torch.randint(1, multi + 1, (B,), device="cuda", generator=g)
            rank = torch.rand((B, n), device="cuda", generator=g).argsort(dim=1).argsort(dim=1)
            lost = rank < e[:, None]
        else:
            which = torch.randint(0, k, (B,), device="cuda", generator=g)
            lost = torch.zeros((B, n), dtype=torch.bool, device="cuda")
            lost[torch.arange(B, device="cuda"), which] = True
        w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
        masks = ((~lost).to(torch.int64) * w).sum(dim=1).to(torch.int32)
        e_d = lost[:, :k].sum(dim=1)
        slots = m   # as a caller that does not scan the masks first
        nbytes = int(((k + e_d) * (e_d > 0)).sum().item()) * L
        if inplace:
            # each route rebuilds its own copy with the erased shards wiped; the copies are compared
            # with the original data (and with each other) afterwards
            wiped = data.clone()
            wiped[lost[:, :k]] = 0x3C
            outs = {r: wiped.clone() for r in routes if r != "direct_oop"}
        else:
            outs = {r: torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda") for r in routes if r != "direct_oop"}

        oop = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda") if "direct_oop" in routes else None

        def dec(r):
            def fn():
                if r == "direct_oop":   # reference: the out-of-place single-slot recover (bench.py's decode)
                    rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S,
                                              masks.data_ptr(), oop.data_ptr(), S, 1, None)
                elif inplace:
                    rc = codec.rs_reconstruct_raw(k, m, L, B, outs[r].data_ptr(), k * S, par.data_ptr(), m * S, S,
                                                  masks.data_ptr(), None, fec.FEC_DEVICE)
                else:
                    rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S,
                                              masks.data_ptr(), outs[r].data_ptr(), slots * S, slots, None)
                assert rc == 0, rc
            return fn

        def timed(fn, iters=5):
            fn()
            s, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e_.record()
            torch.cuda.synchronize()
            return s.elapsed_time(e_) / iters

        name = ("RS(%d,%d) U{1..%d}" % (k, n, multi)) if multi else "RS(%d,%d) one data shard" % (k, n)
        if inplace:
            name += " in place"
        for _ in range(rounds):
            for r in routes:
                old = codec.set_tuning(**ROUTES[r])
                res.setdefault(name, {}).setdefault(r, []).append(timed(dec(r)))
                codec.set_tuning(**old)
        torch.cuda.synchronize()
        cmp = [r for r in routes if r != "direct_oop"]
        same = all(torch.equal(outs[cmp[0]], outs[r]) for r in cmp)
        if inplace:
            same = same and all(torch.equal(outs[r][:, :, :L], data[:, :, :L]) for r in cmp)
        med = {r: round(sorted(v)[len(v) // 2], 4) for r, v in res[name].items()}
        print(json.dumps({"code": name, "blocks": B, "routes_agree": same, "median_ms": med,
                          "TBps": {r: round(nbytes / t / 1e9, 3) for r, t in med.items()}}), flush=True)
        del data, par, outs


if __name__ == "__main__":
    main()
