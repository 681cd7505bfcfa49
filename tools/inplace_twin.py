#!/usr/bin/env python3
"""Diagnostics (round 6): what writing the rebuilt shard in place costs. On bench.py's RS(8,12)
workload (2^20 blocks, one random erased data shard per block, data [B][8][1216] + parity
[B][4][1216]), interleaved in rounds on the same buffers:
  kernel oop      fec_rs_recover_batch, one output slot (the direct kernel; bench.py's decode)
  kernel inplace  fec_rs_reconstruct_batch (the routed kernel's direct body), at route_wpc 3 and 4
  twin oop        fec_probe_recover_traffic into the separate output (the same bytes, no arithmetic)
  twin inplace    the same twin storing into the erased shard's own slot (out == data)
at 3 and 4 workgroups/CU for the twins. Prints median ms and TB/s ((k+1) * 1202 B per block).

usage: inplace_twin.py [--blocks N] [--rounds R]"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=8)
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, B, L, S = 8, 4, args.blocks, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    codec.prepare(k, m)
    data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
    codec.synth_data(0x0FEC, 0, B, k, 1200, data.data_ptr(), k * S, S)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
    masks = torch.empty((B,), dtype=torch.int32, device="cuda")
    erased = torch.empty((B,), dtype=torch.int32, device="cuda")
    codec.synth_single_erasures(0x0FEC, 0, B, k, m, masks.data_ptr(), erased.data_ptr())
    out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    ref = data.clone()
    nbytes = B * (k + 1) * L
    d, p, mk, o = data.data_ptr(), par.data_ptr(), masks.data_ptr(), out.data_ptr()

    def kern_oop():
        assert codec.rs_recover_raw(k, m, L, B, d, k * S, p, m * S, S, mk, o, S, 1, None) == 0

    def kern_inplace(w):
        def fn():
            old = codec.set_tuning(route_wpc=w)
            try:
                assert codec.rs_reconstruct_raw(k, m, L, B, d, k * S, p, m * S, S, mk, None, fec.FEC_DEVICE) == 0
            finally:
                codec.set_tuning(**old)
        return fn

    def twin(w, inplace):
        return lambda: codec.probe_recover_traffic_raw(k, m, L, B, d, k * S, p, m * S, S, mk, d if inplace else o,
                                                       k * S if inplace else S, w)

    forms = {"kernel oop": kern_oop, "kernel inplace wpc3": kern_inplace(3), "kernel inplace wpc4": kern_inplace(4),
             "twin oop wpc3": twin(3, False), "twin oop wpc4": twin(4, False),
             "twin inplace wpc3": twin(3, True), "twin inplace wpc4": twin(4, True)}

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
        for name, fn in forms.items():
            res.setdefault(name, []).append(timed(fn))
    # the kernels rewrite what the twins overwrote: every erased slot in place, and the output
    kern_inplace(4)()
    kern_oop()
    codec.sync()
    rows = torch.arange(B, device="cuda")
    er = erased.long()
    intact = bool(torch.equal(data[:, :, :L], ref[:, :, :L]))
    oop_ok = bool(torch.equal(out[:, 0, :L], ref[rows, er, :L]))
    med = {n: sorted(v)[len(v) // 2] for n, v in res.items()}
    print(json.dumps({"blocks": B, "median_ms": {n: round(v, 4) for n, v in med.items()},
                      "TBps": {n: round(nbytes / (v / 1e3) / 1e12, 3) for n, v in med.items()},
                      "data_intact_after_inplace": intact, "oop_recovered_ok": oop_ok}), flush=True)


if __name__ == "__main__":
    main()
