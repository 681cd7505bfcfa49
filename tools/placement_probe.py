#!/usr/bin/env python3
"""Diagnostics: sensitivity of one decode shape to the relative placement of its buffers. The
data, parity and output regions are carved out of one arena at swept gaps, the same decode is
timed for each placement (median of bursts of 50 launches).

usage: placement_probe.py [--k 2 --m 1 --blocks 65536]"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--blocks", type=int, default=65536)
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    B, k, m, L, S = args.blocks, args.k, args.m, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    nd, npar, no = B * k * S, B * m * S, B * S
    MB = 1 << 20
    arena = torch.zeros(nd + npar + no + 64 * MB, dtype=torch.uint8, device="cuda")
    base = arena.data_ptr()
    erased = torch.randint(0, k, (B,), device="cuda")
    masks = ((1 << (k + m)) - 1 - (1 << erased)).to(torch.int32)
    mp = masks.data_ptr()
    arena[:nd] = torch.randint(0, 256, (nd,), dtype=torch.uint8, device="cuda")

    def timed(fn, n=50):
        fn()
        torch.cuda.synchronize()
        r = []
        for _ in range(5):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(n):
                fn()
            e.record()
            torch.cuda.synchronize()
            r.append(s.elapsed_time(e) / n * 1e3)
        return round(sorted(r)[2], 1)

    res = {}
    for gp in (0, 4096, 65536, MB, 2 * MB + 4096, 7 * MB):
        for go in (0, 4096, 65536, MB, 2 * MB + 4096, 13 * MB):
            dp = base
            pp = base + nd + gp
            op = pp + npar + go

            def enc():
                codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)

            def dec():
                codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S, mp, op, S, 1, None)

            enc()
            res["gap_p=%d gap_o=%d" % (gp, go)] = [timed(enc), timed(dec)]
    v = [x[1] for x in res.values()]
    print(json.dumps({"shape": "RS(%d,%d) x %d" % (k, k + m, B), "encode_decode_us": res,
                      "decode_min_max": [min(v), max(v)]}))


if __name__ == "__main__":
    main()
