#!/usr/bin/env python3
"""Diagnostics: pick the fixed-shape encode form by interleaved A/B in one process (matrix vs
dyadic split-recursive body, flat grid at several residencies, ticket queue), many rounds.
usage: enc_select.py [k,m] [blocks] [only]   (8,4 default; 2^23 / k blocks; only: comma-separated
       substrings of the variant names to keep)"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "8,4").split(","))
    B, L, S = (int(sys.argv[2]) if len(sys.argv) > 2 and int(sys.argv[2]) else (1 << 23) // k), 1202, 1216
    only = [x for x in (sys.argv[3] if len(sys.argv) > 3 else "").split(",") if x]
    codec = fec.Codec(0).use_torch_stream()
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    dp, pp = data.data_ptr(), par.data_ptr()
    variants = {}
    for w in (3, 4, 5):
        variants["matrix flat wpc%d" % w] = dict(enc_queue=0, enc_wpc=w, enc_dyadic=0)
    for w in (0, 3, 4, 5):
        variants["dyadic flat wpc%d" % w] = dict(enc_queue=0, enc_wpc=w, enc_dyadic=1)
    for w in (3, 4):
        variants["dyadic flat wpc%d, plain loads" % w] = dict(enc_queue=0, enc_wpc=w, enc_dyadic=1, enc_nt=2)
    variants["matrix flat wpc3, plain loads"] = dict(enc_queue=0, enc_wpc=3, enc_dyadic=0, enc_nt=2)
    for w in (0, 3):   # shard loads before the table staging (knob enc_early)
        variants["dyadic flat wpc%d early" % w] = dict(enc_queue=0, enc_wpc=w, enc_dyadic=1, enc_early=1)
        variants["matrix flat wpc%d early" % w] = dict(enc_queue=0, enc_wpc=w, enc_dyadic=0, enc_early=1)
    for w in (0, 2, 3):
        variants["bits wpc%d" % w] = dict(enc_queue=0, enc_bits=11, enc_bwpc=w)
        variants["bits stream wpc%d" % w] = dict(enc_queue=0, enc_bits=15, enc_bwpc=w)
    variants["bits wpc0, plain loads"] = dict(enc_queue=0, enc_bits=11, enc_bwpc=0, enc_nt=2)
    if k == 8:
        variants["matrix queue d0 wpc2"] = dict(enc_queue=1, enc_qwpc=2, enc_qdepth=0, enc_dyadic=0)
    if k == 2 and m == 1:   # the [3 2] parity row by one GF doubling per byte, no tables (enc_x23)
        variants["x23"] = dict(enc_queue=0, enc_x23=1)
        variants["x23, plain loads and stores"] = dict(enc_queue=0, enc_x23=1, enc_nt=0)
    if only:
        variants = {n: kv for n, kv in variants.items() if any(x in n for x in only)}
    base = codec.set_tuning(enc_queue=0, enc_wpc=3, enc_qwpc=2, enc_qdepth=0, enc_dyadic=1, enc_nt=3, enc_bits=0,
                            enc_bwpc=0, enc_early=0, enc_x23=0)
    ref = None
    for n, kv in variants.items():   # every form writes the same parity bytes
        codec.set_tuning(**kv)
        par.zero_()
        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)
        torch.cuda.synchronize()
        if ref is None:
            ref = par.clone()
        assert torch.equal(par, ref), n
        codec.set_tuning(**base)
    del ref

    def t(iters=5 if B * k > (1 << 22) else 100):
        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    res = {n: [] for n in variants}
    for _ in range(8):
        for n, kv in variants.items():
            codec.set_tuning(**kv)
            res[n].append(B * (k + m) * L / t() / 1e9)
            codec.set_tuning(**base)
    print(json.dumps({n: [round(sorted(v)[len(v) // 2], 1), round(max(v), 1)] for n, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
