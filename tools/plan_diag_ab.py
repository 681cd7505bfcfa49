#!/usr/bin/env python3
"""Diagnostics: what the plan records cost the multi-erasure decode, interleaved in one process.
Times fec_rs_recover_batch (plan kernel + rebuild) of config_bench's mixes with the plan-form-3
diagnostic knob dec_pdiag (fec_plan.hip; timing only, the plans it makes are wrong): 0 the real
plans, 1 no coefficient rows computed, 2 records copied out as their first 48 bytes, 3 both. The
difference between 0 and 3 bounds what plan records without coefficients could save.

usage: plan_diag_ab.py K M [rounds]"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    k, m = int(sys.argv[1]), int(sys.argv[2])
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    fec = importlib.import_module("0xfec_amd")
    B, L, S, n = 1 << 19, 1202, 1216, k + m
    codec = fec.Codec(0).use_torch_stream()
    g = torch.Generator(device="cuda")
    g.manual_seed(0x0FEC)
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
    e = torch.randint(1, m + 1, (B,), device="cuda", generator=g)
    lost = torch.rand((B, n), device="cuda", generator=g).argsort(dim=1).argsort(dim=1) < e[:, None]
    w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
    masks = ((~lost).to(torch.int64) * w).sum(dim=1).to(torch.int32)
    slots = int(lost[:, :k].sum(dim=1).max().item())
    out = torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda")

    def run():
        rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, masks.data_ptr(),
                                  out.data_ptr(), slots * S, slots, None)
        assert rc == 0

    def t(iters=5):
        run()
        s, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            run()
        e_.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e_) / iters * 1e3

    base = codec.set_tuning(dec_pdiag=0)
    res = {d: [] for d in (0, 1, 2, 3)}
    for _ in range(rounds):
        for d in res:
            codec.set_tuning(dec_pdiag=d)
            res[d].append(t())
    codec.set_tuning(**base)
    print(json.dumps({"shape": "RS(%d,%d) x %d e~U{1..%d}" % (k, n, B, m),
                      "median_us": {"pdiag %d" % d: round(sorted(v)[len(v) // 2], 1) for d, v in res.items()}}))


if __name__ == "__main__":
    main()
