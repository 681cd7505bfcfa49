#!/usr/bin/env python3
"""Diagnostics: per-launch time of one decode shape against the length of the back-to-back burst
it is timed in (does a long burst of short kernels run slower than short bursts?).

usage: burst_probe.py [--k 2 --m 1 --blocks 65536]"""
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
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    erased = torch.randint(0, k, (B,), device="cuda")
    masks = ((1 << (k + m)) - 1 - (1 << erased)).to(torch.int32)
    dp, pp, op, mp = data.data_ptr(), par.data_ptr(), out.data_ptr(), masks.data_ptr()

    def enc():
        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)

    def dec():
        codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S, mp, op, S, 1, None)

    def burst(fn, n):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n * 1e3

    enc()
    res = {}
    for name, fn in (("decode", dec), ("encode", enc)):
        for n in (5, 20, 50, 100, 200):
            res["%s x%d" % (name, n)] = round(sorted(burst(fn, n) for _ in range(5))[2], 1)
    # decode right after a burst of encodes (config_bench's order)
    for _ in range(100):
        enc()
    res["decode x100 after 100 encodes"] = round(burst(dec, 100), 1)
    print(json.dumps({"shape": "RS(%d,%d) x %d" % (k, k + m, B), "median_us": res}))


if __name__ == "__main__":
    main()
