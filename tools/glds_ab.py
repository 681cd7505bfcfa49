#!/usr/bin/env python3
"""Diagnostics (round 6): the RS(8,12) encode with its loads decoupled from its
arithmetic by an LDS-DMA ring (fec_encode.hip rs_encode_glds_kernel, knob enc_glds = D*100 + T, +1000
for its traffic twin) against the shipped flat kernel and the flat traffic twin
(fec_probe_encode_traffic), each at several residencies (knob enc_wpc / the twin's wpc), interleaved
in rounds on the same device buffers in one process (buffer placement moves both by up
to 8 %, so only an interleaved A/B on shared buffers decides). Prints per-form median ms and TB/s
(15.12 GB of algorithmic bytes at 2^20 blocks) and whether every real form wrote the shipped
kernel's parity bytes.

usage: glds_ab.py [--blocks N] [--rounds R] [--iters I] [FORM ...]
  FORM: flat@W | twin@W | glds:DT@W | gtwin:DT@W   (W workgroups per CU, 0 uncapped; DT e.g. 208)
"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

DEFAULT_FORMS = ["flat@3", "flat@2", "twin@2", "twin@3", "gtwin:104@4", "gtwin:208@2", "gtwin:316@1",
                 "glds:104@3", "glds:104@4", "glds:208@2", "glds:216@2", "glds:308@1", "glds:316@1", "glds:416@1"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("forms", nargs="*")
    args = ap.parse_args()
    forms = args.forms or DEFAULT_FORMS
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, B, L, S = 8, 4, args.blocks, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    codec.prepare(k, m)
    data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
    codec.synth_data(0x0FEC, 0, B, k, 1200, data.data_ptr(), k * S, S)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    nbytes = B * (k + m) * L

    def runner(form):
        kind, w = form.split("@")
        w = int(w)
        if kind == "twin":
            return lambda: codec.probe_encode_traffic_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S,
                                                          S, w)
        if kind == "flat":
            knobs = dict(enc_wpc=w, enc_glds=0)
        else:
            dt = int(kind.split(":")[1])
            knobs = dict(enc_wpc=w, enc_glds=dt + (1000 if kind.startswith("gtwin") else 0))

        def fn():
            old = codec.set_tuning(**knobs)
            try:
                codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
            finally:
                codec.set_tuning(**old)
        return fn

    fns = {f: runner(f) for f in forms}
    # bytes: every real form against the shipped kernel
    fns["flat@3"]() if "flat@3" in fns else runner("flat@3")()
    torch.cuda.synchronize()
    ref = par.clone()
    same = {}
    for f, fn in fns.items():
        if f.startswith(("glds", "flat")):
            par.zero_()
            fn()
            torch.cuda.synchronize()
            same[f] = bool(torch.equal(par, ref))
    print(json.dumps({"same_bytes": same}), flush=True)

    def timed(fn):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / args.iters

    res = {}
    for r in range(args.rounds):
        for f, fn in fns.items():
            res.setdefault(f, []).append(timed(fn))
        print(json.dumps({"round": r, "ms": {f: round(v[-1], 4) for f, v in res.items()}}), flush=True)
    med = {f: sorted(v)[len(v) // 2] for f, v in res.items()}
    print(json.dumps({"blocks": B, "median_ms": {f: round(v, 4) for f, v in med.items()},
                      "TBps": {f: round(nbytes / (v / 1e3) / 1e12, 3) for f, v in med.items()},
                      "same_bytes": same}), flush=True)


if __name__ == "__main__":
    main()
