#!/usr/bin/env python3
"""Diagnostics: one library, two or more tuning-knob settings (Codec.set_tuning), interleaved on
the same device buffers in one process, so neither the box nor buffer placement
separates them. Times RS encode and recover (bench.py's shapes: 1202-byte shards, 1216-byte
stride) and compares every setting's output bytes with the first's.

usage: knob_ab.py --k 8 --m 4 [--blocks N] [--multi E (e ~ U{1..E} of n lost; 0: one data
       shard)] [--slots S (output slots; 0: the largest data-loss count)] [--rounds R]
       [--interleaved (one [B][k+m][S] array: parity slots among the data, the batch layer's
       staging layout)] SETTING [SETTING ...]   a SETTING is knob=value[,knob=value...] or "default"
"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse(setting):
    if setting == "default":
        return {}
    return {kv.split("=")[0]: int(kv.split("=")[1]) for kv in setting.split(",")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--multi", type=int, default=0)
    ap.add_argument("--slots", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--interleaved", action="store_true")
    ap.add_argument("settings", nargs="+")
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, B, L, S = args.k, args.m, args.blocks, 1202, 1216
    n = k + m
    codec = fec.Codec(0).use_torch_stream()
    codec.prepare(k, m)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x0FEC)
    if args.interleaved:
        whole = torch.zeros((B, n, S), dtype=torch.uint8, device="cuda")
        codec.synth_data(0x0FEC, 0, B, k, 1200, whole.data_ptr(), n * S, S)
        dptr, pptr, dbs, pbs = whole.data_ptr(), whole.data_ptr() + k * S, n * S, n * S
        data, par = whole, whole[:, k:]
    else:
        data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
        codec.synth_data(0x0FEC, 0, B, k, 1200, data.data_ptr(), k * S, S)
        par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
        dptr, pptr, dbs, pbs = data.data_ptr(), par.data_ptr(), k * S, m * S
    if args.multi:
        e = torch.randint(1, args.multi + 1, (B,), generator=g, device="cuda")
        rank = torch.rand((B, n), generator=g, device="cuda").argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
    else:
        which = torch.randint(0, k, (B,), generator=g, device="cuda")
        lost = torch.zeros((B, n), dtype=torch.bool, device="cuda")
        lost[torch.arange(B, device="cuda"), which] = True
    w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
    masks = ((~lost).to(torch.int64) * w).sum(dim=1).to(torch.int32)
    slots = args.slots or max(1, int(lost[:, :k].sum(dim=1).max().item()))
    out = torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda")
    settings = [parse(s) for s in args.settings]

    def enc():
        codec.rs_encode_raw(k, m, L, B, dptr, dbs, pptr, pbs, S, fec.FEC_DEVICE)

    def rec():
        rc = codec.rs_recover_raw(k, m, L, B, dptr, dbs, pptr, pbs, S, masks.data_ptr(),
                                  out.data_ptr(), slots * S, slots, None)
        assert rc == 0, rc

    def timed(fn):
        fn()
        s, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(args.iters):
            fn()
        e_.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e_) / args.iters

    ref_par = ref_out = None
    same = []
    for kn in settings:
        old = codec.set_tuning(**kn)
        enc()
        rec()
        torch.cuda.synchronize()
        if ref_par is None:
            ref_par, ref_out = par.clone(), out.clone()
            same.append(True)
        else:
            same.append(bool(torch.equal(par, ref_par) and torch.equal(out, ref_out)))
        codec.set_tuning(**old)
    res = {}
    for _ in range(args.rounds):
        for name, kn in zip(args.settings, settings):
            old = codec.set_tuning(**kn)
            res.setdefault(name + " encode", []).append(timed(enc))
            res.setdefault(name + " recover", []).append(timed(rec))
            codec.set_tuning(**old)
    med = {nm: round(sorted(v)[len(v) // 2], 4) for nm, v in res.items()}
    print(json.dumps({"code": "RS(%d,%d)" % (k, n), "blocks": B, "multi": args.multi, "slots": slots,
                      "median_ms": med, "same_bytes": dict(zip(args.settings, same))}), flush=True)


if __name__ == "__main__":
    main()
