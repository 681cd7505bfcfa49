#!/usr/bin/env python3
"""Diagnostics (round 6): the XOR(2,1) reconstruct (fec_xor.hip xor_reconstruct_kernel, the
reference's XOR factory code, config_bench's XOR(2,1) row) by residency, beside its traffic twin
storing in place (the kernel's form) and into a separate buffer. 2^20 blocks of [3][1216] (two
data shards and the parity interleaved, 1202-byte shards), one random erased data shard per block,
interleaved in rounds on the same buffers. Residency is the xor_wpc knob (workgroups per CU; 0 as
many as fit; 6 shipped since round 6). Prints median ms and TB/s (3 * 1202 B per block).
--encode adds the XOR encode and its twin. (The fold A/B of round 6, xor_ab_fold_r06u.log /
_r06v, ran an earlier form of this tool with a temporary knob for each kernel's other fold.)

usage: xor_ab.py [--blocks N] [--rounds R] [--wpc 0,2,3,4,5,6] [--encode]"""
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--wpc", default="0,2,3,4,5,6")
    ap.add_argument("--encode", action="store_true", help="also the XOR encode and its twin")
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, B, L, S = 2, args.blocks, 1202, 1216
    n = k + 1
    codec = fec.Codec(0).use_torch_stream()
    sh = torch.zeros((B, n, S), dtype=torch.uint8, device="cuda")
    codec.synth_data(0x0FEC, 0, B, k, 1200, sh.data_ptr(), n * S, S)
    shp = sh.data_ptr()
    assert fec.lib.fec_xor_encode_batch(codec.handle, k, L, B, shp, n * S, shp + k * S, n * S, S, fec.FEC_DEVICE) == 0
    masks = torch.empty((B,), dtype=torch.int32, device="cuda")
    erased = torch.empty((B,), dtype=torch.int32, device="cuda")
    codec.synth_single_erasures(0x0FEC, 0, B, k, 1, masks.data_ptr(), erased.data_ptr())
    ref = sh.clone()
    out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    mp = masks.data_ptr()
    wpcs = [int(w) for w in args.wpc.split(",")]

    def kern(w):
        def fn():
            old = codec.set_tuning(xor_wpc=w)
            try:
                assert fec.lib.fec_xor_reconstruct_batch(codec.handle, k, L, B, shp, n * S, shp + k * S, n * S, S, mp,
                                                         None, fec.FEC_DEVICE) == 0
            finally:
                codec.set_tuning(**old)
        return fn

    def twin(w, inplace):
        return lambda: codec.probe_recover_traffic_raw(k, 1, L, B, shp, n * S, shp + k * S, n * S, S, mp,
                                                       shp if inplace else out.data_ptr(), n * S if inplace else S, w)

    def enc(w):
        def fn():
            old = codec.set_tuning(xor_wpc=w)
            try:
                assert fec.lib.fec_xor_encode_batch(codec.handle, k, L, B, shp, n * S, shp + k * S, n * S, S,
                                                    fec.FEC_DEVICE) == 0
            finally:
                codec.set_tuning(**old)
        return fn

    def enc_twin(w):
        return lambda: codec.probe_encode_traffic_raw(k, 1, L, B, shp, n * S, shp + k * S, n * S, S, w)

    forms = {}
    for w in wpcs:
        forms["kernel wpc%d" % w] = kern(w)
        forms["twin inplace wpc%d" % w] = twin(w, True)
        forms["twin oop wpc%d" % w] = twin(w, False)
        if args.encode:
            forms["encode wpc%d" % w] = enc(w)
            forms["encode twin wpc%d" % w] = enc_twin(w)

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
    for _ in range(args.rounds):
        for name, fn in forms.items():
            res.setdefault(name, []).append(timed(fn))
    # the twins overwrote the erased slots (the encode forms rewrite the same parity): rebuild
    # them with the shipped kernel and check (the encode twin's parity is not XOR parity: the
    # shipped encode first)
    enc(6)()
    kern(6)()
    codec.sync()
    ok = bool(torch.equal(sh[:, :, :L], ref[:, :, :L]))
    nbytes = B * n * L
    med = {nm: sorted(v)[len(v) // 2] for nm, v in res.items()}
    print(json.dumps({"blocks": B, "median_ms": {nm: round(v, 4) for nm, v in med.items()},
                      "TBps": {nm: round(nbytes / (v / 1e3) / 1e12, 3) for nm, v in med.items()},
                      "rebuilt_ok": ok}), flush=True)


if __name__ == "__main__":
    main()
