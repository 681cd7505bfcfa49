#!/usr/bin/env python3
"""Diagnostics: A/B two builds of lib0xfec_hip.so in ONE process (the process-to-process spread
on a box, 3-5 %, hides kernel changes of that size). Both libraries are loaded side by side
(RTLD_LOCAL), each with its own ctx on the same device and torch stream-free buffers; their
encode and recover calls alternate, many rounds, and the outputs are compared byte for byte.

With --xor: XOR(k,1) encode and in-place reconstruct over the interleaved layout (data shards
then the parity shard per block), one erased data shard per block (--multi > 0: e ~ U{1..multi}
of the k+1 shards; blocks with two or more lost are failures the statuses report).

usage: lib_ab.py LIB_A LIB_B [--k 16 --m 8 --blocks 524288 --multi 8] [--rounds 8] [--xor]"""
import argparse
import ctypes
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib_a")
    ap.add_argument("lib_b")
    ap.add_argument("--k", type=int, default=16)
    ap.add_argument("--m", type=int, default=8)
    ap.add_argument("--blocks", type=int, default=1 << 19)
    ap.add_argument("--multi", type=int, default=8, help="e ~ U{1..multi} erasures over all n shards (0: one data shard)")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--xor", action="store_true")
    ap.add_argument("--no-status", action="store_true", help="--xor timing without a status array")
    args = ap.parse_args()
    if args.xor:
        return xor_main(args)
    import torch
    k, m, B, L, S = args.k, args.m, args.blocks, 1202, 1216
    n = k + m
    g = torch.Generator(device="cuda")
    g.manual_seed(0x0FEC)
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    if args.multi:
        e = torch.randint(1, args.multi + 1, (B,), generator=g, device="cuda")
        rank = torch.rand((B, n), generator=g, device="cuda").argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
    else:
        which = torch.randint(0, k, (B,), generator=g, device="cuda")
        lost = torch.zeros((B, n), dtype=torch.bool, device="cuda")
        lost[torch.arange(B, device="cuda"), which] = True
    w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
    masks = (((~lost).to(torch.int64) * w).sum(dim=1)).to(torch.int32)
    slots = max(1, int(lost[:, :k].sum(dim=1).max().item()))
    outs = [torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda") for _ in range(2)]
    pars = [torch.zeros_like(parity) for _ in range(2)]
    libs, ctxs = [], []
    for path in (args.lib_a, args.lib_b):
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        lib.fec_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
        lib.fec_rs_encode_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                            ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                            ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]
        lib.fec_rs_recover_batch.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                             ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        lib.fec_sync.argtypes = [ctypes.c_void_p]
        ctx = ctypes.c_void_p()
        assert lib.fec_ctx_create(torch.cuda.current_device(), ctypes.byref(ctx)) == 0
        libs.append(lib)
        ctxs.append(ctx)
    FEC_DEVICE = 0   # include/fec_hip.h

    # outputs: each library its own for the byte comparison, then both the same buffers for the
    # timing (where a buffer lands in device memory moves the rate by several %)
    own = [True]

    def enc(i):
        p = pars[i if own[0] else 0]
        rc = libs[i].fec_rs_encode_batch(ctxs[i], k, m, L, B, data.data_ptr(), k * S, p.data_ptr(), m * S, S,
                                         FEC_DEVICE)
        assert rc == 0, rc

    def rec(i):
        o = outs[i if own[0] else 0]
        rc = libs[i].fec_rs_recover_batch(ctxs[i], k, m, L, B, data.data_ptr(), k * S, pars[0].data_ptr(), m * S, S,
                                          masks.data_ptr(), o.data_ptr(), slots * S, slots, None, FEC_DEVICE)
        assert rc == 0, rc

    for i in (0, 1):
        enc(i)
        assert libs[i].fec_sync(ctxs[i]) == 0
    assert torch.equal(pars[0], pars[1]), "encode outputs differ"
    for i in (0, 1):
        rec(i)
        rcs = libs[i].fec_sync(ctxs[i])
        assert rcs == 0 or (rcs == -4 and args.multi > m), rcs   # too few shards in some blocks
    assert torch.equal(outs[0], outs[1]), "recover outputs differ"
    own[0] = False

    def t(fn, i):
        fn(i)
        libs[i].fec_sync(ctxs[i])
        s, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the library runs on its own stream: bracket with device-wide synchronisation
        torch.cuda.synchronize()
        s.record()
        for _ in range(args.iters):
            fn(i)
        libs[i].fec_sync(ctxs[i])
        e_.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e_) / args.iters

    res = {"encode A": [], "encode B": [], "recover A": [], "recover B": []}
    for _ in range(args.rounds):
        for i, nm in ((0, "A"), (1, "B")):
            res["encode " + nm].append(t(enc, i))
            res["recover " + nm].append(t(rec, i))
    med = {kk: sorted(v)[len(v) // 2] for kk, v in res.items()}
    print(json.dumps({"shape": "RS(%d,%d) x %d, multi %d" % (k, n, B, args.multi),
                      "median_ms": {kk: round(v, 4) for kk, v in med.items()},
                      "B/A": {"encode": round(med["encode B"] / med["encode A"], 4),
                              "recover": round(med["recover B"] / med["recover A"], 4)}}))


def xor_main(args):
    import torch
    k, B, L, S = args.k, args.blocks, 1202, 1216
    n = k + 1
    g = torch.Generator(device="cuda")
    g.manual_seed(0x0FEC)
    base = torch.zeros((B, n, S), dtype=torch.uint8, device="cuda")
    base[:, :k, :L] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device="cuda", generator=g)
    if args.multi:
        e = torch.randint(1, args.multi + 1, (B,), generator=g, device="cuda")
        rank = torch.rand((B, n), generator=g, device="cuda").argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
    else:
        which = torch.randint(0, k, (B,), generator=g, device="cuda")
        lost = torch.zeros((B, n), dtype=torch.bool, device="cuda")
        lost[torch.arange(B, device="cuda"), which] = True
    w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
    masks = (((~lost).to(torch.int64) * w).sum(dim=1)).to(torch.int32)
    shs = [base.clone() for _ in range(2)]
    sts = [torch.zeros((B,), dtype=torch.int32, device="cuda") for _ in range(2)]
    libs, ctxs = [], []
    vp, sz, i_ = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    for path in (args.lib_a, args.lib_b):
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        lib.fec_ctx_create.argtypes = [i_, ctypes.POINTER(vp)]
        lib.fec_xor_encode_batch.argtypes = [vp, i_, sz, sz, vp, sz, vp, sz, sz, i_]
        lib.fec_xor_reconstruct_batch.argtypes = [vp, i_, sz, sz, vp, sz, vp, sz, sz, vp, vp, i_]
        lib.fec_sync.argtypes = [vp]
        ctx = vp()
        assert lib.fec_ctx_create(torch.cuda.current_device(), ctypes.byref(ctx)) == 0
        libs.append(lib)
        ctxs.append(ctx)
    FEC_DEVICE = 0

    # each library its own buffers for the byte comparison, then both the same ones for the timing
    # (as in the RS mode)
    own = [True]

    def enc(i):
        p = shs[i if own[0] else 0].data_ptr()
        assert libs[i].fec_xor_encode_batch(ctxs[i], k, L, B, p, n * S, p + k * S, n * S, S, FEC_DEVICE) == 0

    use_status = [True]

    def rec(i):
        p = shs[i if own[0] else 0].data_ptr()
        st = sts[i if own[0] else 0].data_ptr() if use_status[0] else None
        assert libs[i].fec_xor_reconstruct_batch(ctxs[i], k, L, B, p, n * S, p + k * S, n * S, S, masks.data_ptr(),
                                                 st, FEC_DEVICE) == 0

    for i in (0, 1):
        enc(i)
        libs[i].fec_sync(ctxs[i])
    torch.cuda.synchronize()
    assert torch.equal(shs[0], shs[1]), "encode outputs differ"
    ref = shs[0].clone()
    for i in (0, 1):
        shs[i][lost[:, :, None].expand(-1, -1, S) & (torch.arange(n, device="cuda") < k)[None, :, None]] = 0
        torch.cuda.synchronize()   # the library runs on its own stream
        rec(i)
        rcs = libs[i].fec_sync(ctxs[i])
        assert rcs in (0, -4), rcs
    for i, nm in ((0, "A"), (1, "B")):
        good = sts[i] == 0
        bad = (shs[i][good, :k, :L] != ref[good, :k, :L]).flatten(1).any(dim=1)
        if bad.any():
            rows = torch.nonzero(good).flatten()[torch.nonzero(bad).flatten()[:8]].tolist()
            raise AssertionError("%s: %d blocks reconstructed wrong, e.g. %s" % (nm, int(bad.sum()), rows))
    assert torch.equal(sts[0], sts[1]), "statuses differ"
    assert torch.equal(shs[0], shs[1]), "reconstruct outputs differ"
    use_status[0] = not args.no_status
    own[0] = False

    def t(fn, i):
        fn(i)
        libs[i].fec_sync(ctxs[i])
        s, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(args.iters):
            fn(i)
        libs[i].fec_sync(ctxs[i])
        e_.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e_) / args.iters

    res = {"encode A": [], "encode B": [], "recover A": [], "recover B": []}
    for _ in range(args.rounds):
        for i, nm in ((0, "A"), (1, "B")):
            res["encode " + nm].append(t(enc, i))
            res["recover " + nm].append(t(rec, i))
    med = {kk: sorted(v)[len(v) // 2] for kk, v in res.items()}
    print(json.dumps({"shape": "XOR(%d,%d) x %d, multi %d, status %s" % (k, n, B, args.multi, use_status[0]),
                      "median_ms": {kk: round(v, 4) for kk, v in med.items()},
                      "B/A": {"encode": round(med["encode B"] / med["encode A"], 4),
                              "recover": round(med["recover B"] / med["recover A"], 4)}}))


if __name__ == "__main__":
    main()
