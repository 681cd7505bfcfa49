#!/usr/bin/env python3
"""Diagnostics: the RS(8,12) single-erasure decode (fec_rs_recover_batch, the bench's decode) and
traffic twins of its access shape (tools/dec_twin_probe.hip) at every residency, in interleaved
bursts in one process, on the bench's buffers (data [B][8][1216], parity [B][4][1216], recovered
[B][1216], one erased data shard per block from the device generator).

Twin modes: vec (the kernel's vector mask load in front of the shard loads), free (no mask load:
addresses known at launch), scalar (masks by scalar loads), read8 (the block's 8 data shards + one
store: no holes, no parity region). Each mode as a pure-traffic twin (xor) and with the decode's
field arithmetic (arith). Rates are algorithmic bytes (9 shards of 1202 B per block) / time.

With --multi: the RS(16,24) multi-erasure decode instead (2^19 blocks), every block with one
erasure pattern (3 data + 2 parity shards lost: 16 reads + 3 stores), against rebuild twins whose
present mask arrives by a per-lane vector load, by scalar loads, as a kernel argument (addresses
known at launch) or through the rebuild's plan-record staging (a record per block, vector-loaded
into LDS); and the library's decode of the config #4 distribution (e ~ U{1..8} of 24) beside it.

usage: dec_twin_probe.py [blocks] [rounds] [--multi] [--rebuild (recompile the probe)] [--build-only]"""
import ctypes
import importlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
SO = os.path.join(HERE, "libdec_twin_probe.so")


def main():
    if not os.path.exists(SO) or "--rebuild" in sys.argv:
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                               os.path.join(HERE, "dec_twin_probe.hip")])
    if "--build-only" in sys.argv:
        return
    if "--multi" in sys.argv:
        return rebuild_main()
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 1 << 20
    rounds = int(args[1]) if len(args) > 1 else 7
    import torch
    fec = importlib.import_module("0xfec_amd")
    lib = ctypes.CDLL(SO)
    vp, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.dec_probe.argtypes = [i, i, i, vp, vp, vp, vp, sz, sz, sz, sz, u, u, vp]
    k, m, L, S = 8, 4, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    codec.prepare(k, m)
    st = torch.cuda.current_stream().cuda_stream
    data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
    codec.synth_data(0x0FEC, 0, B, k, 1200, data.data_ptr(), k * S, S)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    masks = torch.empty((B,), dtype=torch.int32, device="cuda")
    erased = torch.empty((B,), dtype=torch.int32, device="cuda")
    codec.synth_single_erasures(0x0FEC, 0, B, k, m, masks.data_ptr(), erased.data_ptr())
    rec = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
    nbytes = B * (k + 1) * L

    def lib_decode():
        rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, masks.data_ptr(),
                                  rec.data_ptr(), S, 1, None)
        assert rc == 0, rc

    def probe(mode, arith, wpc):
        def fn():
            rc = lib.dec_probe(mode, arith, wpc, data.data_ptr(), par.data_ptr(), rec.data_ptr(), masks.data_ptr(),
                               k * S, m * S, S, S, L, B, st)
            assert rc == 0, rc
        return fn

    def timed(fn, iters=4):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    # correctness of the library path on these buffers (the erased shard comes back)
    lib_decode()
    torch.cuda.synchronize()
    rows = torch.arange(B, device="cuda")
    ok = bool(torch.equal(rec[:, 0, :L], data[rows, erased.long(), :L]))
    modes = {"vec": 0, "free": 1, "scalar": 2, "read8": 3}
    base = codec.set_tuning(dir_wpc=-1)
    res = {}
    print("probe start B=%d rounds=%d decode_ok=%s" % (B, rounds, ok), flush=True)
    for r in range(rounds):
        for w in (2, 3, 4, 5, 0):
            codec.set_tuning(dir_wpc=w)
            lib_decode()
            res.setdefault("decode wpc%d" % w, []).append(nbytes / timed(lib_decode) / 1e12)
            for name, md in modes.items():
                for arith in (0, 1):
                    fn = probe(md, arith, w)
                    fn()
                    res.setdefault("%s %s wpc%d" % (name, "arith" if arith else "xor", w), []).append(
                        nbytes / timed(fn) / 1e12)
        print("round %d done" % r, flush=True)
    codec.set_tuning(**base)
    med = {n: round(sorted(v)[len(v) // 2], 3) for n, v in res.items()}
    print(json.dumps({"blocks": B, "rounds": rounds, "decode_ok": ok, "TBps_median": med}, indent=1), flush=True)


def rebuild_main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B = int(args[0]) if args else 1 << 19
    rounds = int(args[1]) if len(args) > 1 else 7
    import torch
    fec = importlib.import_module("0xfec_amd")
    lib = ctypes.CDLL(SO)
    vp, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.rebuild_probe.argtypes = [i, i, vp, vp, vp, vp, vp, u, sz, sz, sz, sz, u, u, vp]
    k, m, L, S, n = 16, 8, 1202, 1216, 24
    codec = fec.Codec(0).use_torch_stream()
    codec.prepare(k, m)
    st = torch.cuda.current_stream().cuda_stream
    data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
    codec.synth_data(0x0FEC, 0, B, k, 1200, data.data_ptr(), k * S, S)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, fec.FEC_DEVICE)
    lost = (1, 7, 12, 17, 20)                  # data 1, 7, 12; parity 1, 4
    cmask = ((1 << n) - 1) & ~sum(1 << x for x in lost)
    masks = torch.full((B,), cmask, dtype=torch.int32, device="cuda")
    recs = torch.zeros((B, 40), dtype=torch.int32, device="cuda")
    recs[:, 0] = cmask
    out = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(0x1624)
    e = torch.randint(1, m + 1, (B,), device="cuda", generator=g)
    rank = torch.rand((B, n), device="cuda", generator=g).argsort(dim=1).argsort(dim=1)
    lostu = rank < e[:, None]
    w = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"), torch.arange(n, device="cuda"))
    masks_u = ((~lostu).to(torch.int64) * w).sum(dim=1).to(torch.int32)
    bytes_c = B * (k + 3) * L
    bytes_u = int(((k + lostu[:, :k].sum(dim=1)) * (lostu[:, :k].sum(dim=1) > 0)).sum().item()) * L

    def lib_decode(mk):
        def fn():
            rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, mk.data_ptr(),
                                      out.data_ptr(), m * S, m, None)
            assert rc == 0, rc
        return fn

    def probe(mode, wpc):
        def fn():
            rc = lib.rebuild_probe(mode, wpc, data.data_ptr(), par.data_ptr(), out.data_ptr(), masks.data_ptr(),
                                   recs.data_ptr(), cmask, k * S, m * S, S, m * S, L, B, st)
            assert rc == 0, rc
        return fn

    def timed(fn, iters=3):
        fn()
        s, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e_.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e_) / iters / 1e3

    lib_decode(masks)()
    torch.cuda.synchronize()
    ok = all(bool(torch.equal(out[:, r, :L], data[:, x, :L])) for r, x in enumerate((1, 7, 12)))
    base = codec.set_tuning(dec_wpc=0)
    res = {}
    print("rebuild probe start B=%d rounds=%d decode_ok=%s" % (B, rounds, ok), flush=True)
    names = {0: "vecmask", 1: "scalarmask", 2: "constmask", 3: "record"}
    for r in range(rounds):
        for wp in (2, 3, 4, 5, 0):
            codec.set_tuning(dec_wpc=wp)
            res.setdefault("decode 1pattern wpc%d" % wp, []).append(bytes_c / timed(lib_decode(masks)) / 1e12)
            res.setdefault("decode U1..8 wpc%d" % wp, []).append(bytes_u / timed(lib_decode(masks_u)) / 1e12)
            for md, nm in names.items():
                res.setdefault("%s wpc%d" % (nm, wp), []).append(bytes_c / timed(probe(md, wp)) / 1e12)
        print("round %d done" % r, flush=True)
    codec.set_tuning(**base)
    med = {nm: round(sorted(v)[len(v) // 2], 3) for nm, v in res.items()}
    print(json.dumps({"blocks": B, "rounds": rounds, "decode_ok": ok, "TBps_median": med}, indent=1), flush=True)


if __name__ == "__main__":
    main()
