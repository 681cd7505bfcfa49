#!/usr/bin/env python3
"""Diagnostics: RS decode routes on mixed-erasure batches of the small codes (those the direct
single-erasure kernel serves by default: k*m*k PermTabs <= 16 KiB). Each code runs a batch with
e ~ U{1..m} losses uniform over all n shards (every block recoverable), one output slot per
possible data loss, through the default route (direct kernel + hard worklist), the sorted-plan
wave route (knob dec_direct=0) and the tile route (dec_direct=0, dec_wave=0), interleaved in one
process; the outputs of the routes are compared byte for byte.

usage: mixed_route_probe.py [blocks] [rounds]"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

L, S = 1202, 1216
ROUTES = {"default": {}, "wave": {"dec_direct": 0}, "tile": {"dec_direct": 0, "dec_wave": 0}}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 1 << 18
    rounds = int(args[1]) if len(args) > 1 else 5
    import torch
    fec = importlib.import_module("0xfec_amd")
    codec = fec.Codec(0).use_torch_stream()
    res = {}
    for k, m, multi in ((8, 4, 4), (8, 4, 2), (10, 4, 4), (4, 2, 2), (2, 2, 2)):
        n = k + m
        codec.prepare(k, m)
        g = torch.Generator(device="cuda")
        g.manual_seed(0x0FEC + k)
        data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda", generator=g)
        par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
        codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
        e = torch.randint(1, multi + 1, (B,), device="cuda", generator=g)
        rank = torch.rand((B, n), device="cuda", generator=g).argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
        w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
        masks = ((~lost).to(torch.int64) * w).sum(dim=1).to(torch.int32)
        e_d = lost[:, :k].sum(dim=1)
        slots = max(1, int(e_d.max().item()))
        nbytes = int(((k + e_d) * (e_d > 0)).sum().item()) * L
        outs = {r: torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda") for r in ROUTES}

        def dec(r):
            def fn():
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

        name = "RS(%d,%d) U{1..%d}" % (k, n, multi)
        for _ in range(rounds):
            for r, knobs in ROUTES.items():
                old = codec.set_tuning(**knobs)
                res.setdefault(name, {}).setdefault(r, []).append(timed(dec(r)))
                codec.set_tuning(**old)
        torch.cuda.synchronize()
        same = all(torch.equal(outs["default"], outs[r]) for r in ROUTES)
        med = {r: round(sorted(v)[len(v) // 2], 4) for r, v in res[name].items()}
        print(json.dumps({"code": name, "blocks": B, "routes_agree": same, "median_ms": med,
                          "TBps": {r: round(nbytes / t / 1e9, 3) for r, t in med.items()}}), flush=True)
        del data, par, outs


if __name__ == "__main__":
    main()
