#!/usr/bin/env python3
"""Diagnostics: pick the RS(8,12) encode launch form by interleaved A/B in one process
(flat fixed-shape grid at several residencies vs the ticket-queue kernel), many rounds."""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    fec = importlib.import_module("0xfec_amd")
    B, k, m, L, S = 1 << 20, 8, 4, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    dp, pp = data.data_ptr(), par.data_ptr()
    variants = {
        "flat wpc0": dict(enc_queue=0, enc_wpc=0), "flat wpc3": dict(enc_queue=0, enc_wpc=3),
        "flat wpc4": dict(enc_queue=0, enc_wpc=4), "flat wpc5": dict(enc_queue=0, enc_wpc=5),
        "queue d0 wpc2": dict(enc_queue=1, enc_qwpc=2, enc_qdepth=0),
        "queue d0 wpc3": dict(enc_queue=1, enc_qwpc=3, enc_qdepth=0),
        "queue d1 wpc2": dict(enc_queue=1, enc_qwpc=2, enc_qdepth=1),
    }
    base = codec.set_tuning(enc_queue=1, enc_wpc=3, enc_qwpc=2, enc_qdepth=0)

    def t(iters=5):
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
