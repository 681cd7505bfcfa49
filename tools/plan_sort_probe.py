#!/usr/bin/env python3
"""Diagnostics: run the multi-erasure recover of config_bench's mixes (RS(16,24) U{1..8},
RS(20,30) U{1..10}) with one plan-sort window (knob dec_psort), for rocprofv3 --kernel-trace
--stats to split the time between the sorted plan kernel and the rebuild.
usage: plan_sort_probe.py K M MULTI PSORT [iters] [knob=value ...]"""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    k, m, multi, psort = (int(x) for x in sys.argv[1:5])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    fec = importlib.import_module("0xfec_amd")
    B, L, S, n = 1 << 19, 1202, 1216, k + m
    codec = fec.Codec(0).use_torch_stream()
    codec.set_tuning(dec_psort=psort, **{kv.split("=")[0]: int(kv.split("=")[1]) for kv in sys.argv[6:]})
    g = torch.Generator(device="cuda")
    g.manual_seed(0x0FEC)
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda", generator=g)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
    e = torch.randint(1, multi + 1, (B,), device="cuda", generator=g)
    lost = torch.rand((B, n), device="cuda", generator=g).argsort(dim=1).argsort(dim=1) < e[:, None]
    w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
    masks = ((~lost).to(torch.int64) * w).sum(dim=1).to(torch.int32)
    slots = int(lost[:, :k].sum(dim=1).max().item())
    out = torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda")
    for _ in range(iters):
        rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, masks.data_ptr(),
                                  out.data_ptr(), slots * S, slots, None)
        assert rc == 0
    codec.sync()
    print("ok", k, m, multi, psort)


if __name__ == "__main__":
    main()
