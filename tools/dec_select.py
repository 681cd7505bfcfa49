#!/usr/bin/env python3
"""Diagnostics: pick the RS(8,12) single-erasure recover launch form by interleaved A/B in one
process (wave vs tile reconstruct, residency caps, XCD order), many rounds."""
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
    par = torch.randint(0, 256, (B, m, S), dtype=torch.uint8, device="cuda")
    out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    erased = torch.randint(0, k, (B,), device="cuda")
    masks = ((1 << (k + m)) - 1 - (1 << erased)).to(torch.int32)
    dp, pp, op = data.data_ptr(), par.data_ptr(), out.data_ptr()
    variants = {"wave + plan kernel": dict(dec_wave=1, dec_fused=0, dec_wpc=0, dec_swz=0, dec_ipl=1),
                "ipl2 + plan kernel": dict(dec_wave=1, dec_fused=0, dec_wpc=0, dec_swz=0, dec_ipl=2),
                "ipl2 fused": dict(dec_wave=1, dec_fused=1, dec_wpc=0, dec_swz=0, dec_ipl=2),
                "ipl2 swz": dict(dec_wave=1, dec_fused=0, dec_wpc=0, dec_swz=1, dec_ipl=2)}
    for w in (2, 3, 4):
        variants["ipl2 wpc%d" % w] = dict(dec_wave=1, dec_fused=0, dec_wpc=w, dec_swz=0, dec_ipl=2)
        variants["ipl2 wpc%d swz" % w] = dict(dec_wave=1, dec_fused=0, dec_wpc=w, dec_swz=1, dec_ipl=2)
    base = codec.set_tuning(dec_wave=1, dec_fused=0, dec_wpc=0, dec_swz=0, dec_ipl=1)

    def run():
        codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S, masks.data_ptr(), op, S, 1, None)

    def t(iters=5):
        run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            run()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    run()
    torch.cuda.synchronize()
    run_ref = out.clone()
    for n, kv in variants.items():
        codec.set_tuning(**kv)
        out.zero_()
        run()
        torch.cuda.synchronize()
        assert torch.equal(out, run_ref), n
        codec.set_tuning(**base)
    res = {n: [] for n in variants}
    for _ in range(8):
        for n, kv in variants.items():
            codec.set_tuning(**kv)
            res[n].append(B * (k + 1) * L / t() / 1e9)
            codec.set_tuning(**base)
    print(json.dumps({n: [round(sorted(v)[len(v) // 2], 1), round(max(v), 1)] for n, v in res.items()}))


if __name__ == "__main__":
    main()
