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
    D = dict(dec_wave=1, dec_fused=0, dec_wpc=0, dec_swz=1, dec_ipl=0)
    # name -> (tuning, output slots per block: the recover plans min(k, m, slots) rows). With
    # one erasure per block only slot 0 is written, so the 4-slot runs use the same one-slot
    # buffer (block stride S): identical stores, only the planned row count differs.
    variants = {"wave, 1 slot": (dict(D, dec_swz=0), 1),
                "wave, 4 slots": (dict(D, dec_swz=0), 4),
                "wave swz, 1 slot (default)": (D, 1),
                "wave swz, 4 slots": (D, 4),
                "wave fused swz, 1 slot": (dict(D, dec_fused=1, dec_swz=1), 1),
                "wave ipl2 swz, 1 slot": (dict(D, dec_ipl=2, dec_swz=1), 1)}
    for w in (4, 5, 6):
        variants["wave swz wpc%d, 1 slot" % w] = (dict(D, dec_swz=1, dec_wpc=w), 1)
    for w in (0, 4, 5):
        variants["wave swz seq2 wpc%d, 1 slot" % w] = (dict(D, dec_ipl=3, dec_wpc=w), 1)
    # diagnostics (wrong output): every wave stages block 0's plan, an L2-resident load
    variants["DIAG shared plan"] = (dict(D, dec_diag=1), 1)
    variants["DIAG shared plan wpc4"] = (dict(D, dec_diag=1, dec_wpc=4), 1)
    base = codec.set_tuning(**D)

    def run(slots=1):
        codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S, masks.data_ptr(), op, S, slots, None)

    def t(slots, iters=5):
        run(slots)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            run(slots)
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    run()
    torch.cuda.synchronize()
    ref = out.clone()
    for n, (kv, slots) in variants.items():
        codec.set_tuning(**kv)
        out.zero_()
        run(slots)
        torch.cuda.synchronize()
        assert n.startswith("DIAG") or torch.equal(out, ref), n
        codec.set_tuning(**base)
    res = {n: [] for n in variants}
    for _ in range(8):
        for n, (kv, slots) in variants.items():
            codec.set_tuning(**kv)
            res[n].append(B * (k + 1) * L / t(slots) / 1e9)
            codec.set_tuning(**base)
    print(json.dumps({n: [round(sorted(v)[len(v) // 2], 1), round(max(v), 1)] for n, v in res.items()}))


if __name__ == "__main__":
    main()
