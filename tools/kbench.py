#!/usr/bin/env python3
"""Kernel-level A/B bench (diagnostics, not the contract bench): times each codec kernel on
one resident RS(8,12)-shaped batch, interleaved over rounds in one process, beside a torch
copy of the same byte count for the box's achievable HBM rate."""
import argparse
import ctypes
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--enc", default="3:0:1,2:0:1,1:0:1,0:0:1",
                    help="encode nt:grid_mult:items_per_thread (grid_mult 0 -> 1 with ipt)")
    ap.add_argument("--dec", default="3:8:0:1,2:8:0:1",
                    help="decode nt:rounds:grid_mult:tiles_per_wg")
    ap.add_argument("--xor", default="0:1", help="xor grid_mult:items_per_thread")
    ap.add_argument("--occ", default="",
                    help="swz:enc_wpc:dec_wpc triples; when given, only the split-layout encode and "
                         "recover (the bench.py step) are timed, once per triple")
    ap.add_argument("--dsweep", default="",
                    help="wave:dec_swz:dec_wpc triples; when given, only the split-layout recover "
                         "(the bench.py decode) is timed, once per triple")
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    fec.lib.fec__set_tuning.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    B, k, m = args.blocks, args.k, args.m
    n, L, S = k + m, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    sh = torch.randint(0, 256, (B, n, S), dtype=torch.uint8, device="cuda")
    erased = torch.randint(0, k, (B,), device="cuda")
    masks = ((1 << n) - 1 - (1 << erased)).to(torch.int32)
    base, bs = sh.data_ptr(), n * S
    cp_src = torch.empty(B * k * S, dtype=torch.uint8, device="cuda")
    cp_dst = torch.empty(B * m * S, dtype=torch.uint8, device="cuda")
    rd = torch.empty(B * (k + m) * S // 4, dtype=torch.int32, device="cuda")

    def t(fn):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        torch.cuda.synchronize()
        s.record()
        for _ in range(args.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / args.iters

    def tune(**kv):
        keys = {"enc_nt": 0, "dec_nt": 1, "grid_mult": 2, "dec_max_rounds": 3, "pad_zero": 4,
                "items_per_thread": 5, "tiles_per_wg": 6, "rotate": 7, "xcd_swz": 8, "enc_wpc": 9,
                "dec_wpc": 10, "enc_fixed": 11, "dec_swz": 12, "gen_wpc": 13,
                "enc_queue": 14, "enc_qwpc": 15, "enc_qdepth": 16, "dec_wave": 17}
        for key, val in kv.items():
            fec.lib.fec__set_tuning(codec.handle, keys[key], val)

    def enc(v, g, ipt):
        def f():
            tune(enc_nt=v, grid_mult=max(g, 1), items_per_thread=ipt, pad_zero=1)
            codec.rs_encode_raw(k, m, L, B, base, bs, base + k * S, bs, S, fec.FEC_DEVICE)
        return f

    def dec(nt, rounds, g, tpw):
        def f():
            tune(dec_nt=nt, dec_max_rounds=rounds, grid_mult=max(g, 1), tiles_per_wg=tpw, pad_zero=1)
            codec.rs_reconstruct_raw(k, m, L, B, base, bs, base + k * S, bs, S, masks.data_ptr(), None,
                                     fec.FEC_DEVICE)
        return f

    def xor(g, ipt):
        def f():
            tune(grid_mult=max(g, 1), items_per_thread=ipt, pad_zero=1)
            fec.lib.fec_xor_encode_batch(codec.handle, k, L, B, base, bs, base + k * S, bs, S, fec.FEC_DEVICE)
        return f

    dsplit = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    psplit = torch.randint(0, 256, (B, m, S), dtype=torch.uint8, device="cuda")

    def enc_split(pol, rot=1):
        def f():
            tune(enc_nt=pol, grid_mult=1, items_per_thread=1, pad_zero=1, rotate=rot)
            codec.rs_encode_raw(k, m, L, B, dsplit.data_ptr(), k * S, psplit.data_ptr(), m * S, S, fec.FEC_DEVICE)
        return f

    def dec_split(nt):
        def f():
            tune(dec_nt=nt, dec_max_rounds=8, grid_mult=1, tiles_per_wg=1, pad_zero=1)
            codec.rs_reconstruct_raw(k, m, L, B, dsplit.data_ptr(), k * S, psplit.data_ptr(), m * S, S,
                                     masks.data_ptr(), None, fec.FEC_DEVICE)
        return f

    outb = torch.empty((B, 1, S), dtype=torch.uint8, device="cuda")

    def rec_split(pol, rot=1):
        def f():
            tune(dec_nt=pol, dec_max_rounds=8, grid_mult=1, tiles_per_wg=1, pad_zero=1, rotate=rot)
            codec.rs_recover_raw(k, m, L, B, dsplit.data_ptr(), k * S, psplit.data_ptr(), m * S, S,
                                 masks.data_ptr(), outb.data_ptr(), S, 1, None)
        return f

    cases = {}
    if args.dsweep:
        args.occ = ""
        for spec in args.dsweep.split(","):
            wv, dsw, dw = [int(x) for x in spec.split(":")]

            def dsw_case(fn, wv=wv, dsw=dsw, dw=dw):
                def f():
                    tune(dec_wave=wv, dec_swz=dsw, dec_wpc=dw)
                    fn()
                return f
            cases["rs_recover split wave%d swz%d wpc%d" % (wv, dsw, dw)] = (dsw_case(rec_split(3, 0)), B * (k + 1) * L)
    if args.occ:
        # spec = swz:enc_wpc:dec_swz:dec_wpc:enc_fixed[:queue_wpc[:depth]]  (queue_wpc 0: flat grid)
        for spec in args.occ.split(","):
            v = [int(x) for x in spec.split(":")] + [0, 1]
            swz, ew, dsw, dw, fx, qw, qd = v[:7]

            def occ(fn, swz=swz, ew=ew, dsw=dsw, dw=dw, fx=fx, qw=qw, qd=qd):
                def f():
                    tune(xcd_swz=swz, enc_wpc=ew, dec_swz=dsw, dec_wpc=dw, enc_fixed=fx,
                         enc_queue=1 if qw else 0, enc_qwpc=max(qw, 1), enc_qdepth=qd)
                    fn()
                return f
            cases["rs_encode split fixed%d swz%d wpc%d queue%d d%d" % (fx, swz, ew, qw, qd)] = (
                occ(enc_split(3, 0)), B * n * L)
            if not qw:
                cases["rs_recover split swz%d wpc%d" % (dsw, dw)] = (occ(rec_split(3, 0)), B * (k + 1) * L)
    for rot in (1, 0) if not (args.occ or args.dsweep) else ():
        cases["rs_recover split rot%d" % rot] = (rec_split(3, rot), B * (k + 1) * L)
        cases["rs_encode split rot%d" % rot] = (enc_split(3, rot), B * n * L)
    if not (args.occ or args.dsweep):
        cases["rs_reconstruct split pol3"] = (dec_split(3), B * (k + 1) * L)
    for spec in [x for x in args.enc.split(",") if x and not (args.occ or args.dsweep)]:
        v, g, ipt = [int(x) for x in spec.split(":")]
        cases["rs_encode nt%d g%d ipt%d" % (v, g, ipt)] = (enc(v, g, ipt), B * n * L)
    for spec in [x for x in args.dec.split(",") if x and not (args.occ or args.dsweep)]:
        nt, r, g, tpw = [int(x) for x in spec.split(":")]
        cases["rs_reconstruct nt%d r%d g%d tpw%d" % (nt, r, g, tpw)] = (dec(nt, r, g, tpw), B * (k + 1) * L)
    for spec in [x for x in args.xor.split(",") if x and not (args.occ or args.dsweep)]:
        g, ipt = [int(x) for x in spec.split(":")]
        cases["xor_encode_k%d g%d ipt%d" % (k, g, ipt)] = (xor(g, ipt), B * (k + 1) * L)
    cases["torch_copy_%dto%d" % (k, m)] = (lambda: cp_dst.copy_(cp_src[:cp_dst.numel()]), 2 * cp_dst.numel())
    cases["torch_sum_read"] = (lambda: rd.sum(), rd.numel() * 4)
    if args.occ:
        # the fixed-shape encode must equal the generic one byte for byte
        tune(enc_fixed=0, enc_queue=0)
        enc_split(3, 0)()
        torch.cuda.synchronize()
        ref = psplit.clone()
        psplit.zero_()
        for q, d in ((0, 1), (1, 1), (1, 2)):
            psplit.zero_()
            tune(enc_fixed=1, enc_queue=q, enc_qwpc=2, enc_qdepth=d)
            enc_split(3, 0)()
            torch.cuda.synchronize()
            print("fixed encode (queue=%d depth=%d) == generic encode:" % (q, d),
                  bool(torch.equal(ref[:, :, :L], psplit[:, :, :L])), flush=True)
        del ref
    res = {name: [] for name in cases}
    for _ in range(args.rounds):
        for name, (fn, nbytes) in cases.items():
            ms = t(fn)
            res[name].append(nbytes / (ms / 1e3) / 1e9)
    out = {name: {"GB/s_median": round(sorted(v)[len(v) // 2], 1), "GB/s_max": round(max(v), 1)} for name, v in res.items()}
    print(json.dumps({"blocks": B, "k": k, "m": m, "results": out}, indent=1))


if __name__ == "__main__":
    main()
