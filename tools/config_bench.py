#!/usr/bin/env python3
"""Device-resident encode + decode rates for every GPU configuration of BASELINE.json
(diagnostics beside bench.py, which times only the headline RS(8,12) config).

  RS(2,3)    65 536 blocks, one random erased data shard per block
  RS(8,12)   2^20 blocks, one random erased data shard per block (bench.py's workload)
  RS(16,24)  2^19 blocks, e ~ U{1..8} erasures per block, uniform over all 24 shards
  XOR(2,1)   2^20 blocks (the reference's XOR factory code), one erased data shard
  RS(20,30)  2^19 blocks (the reference's RS factory code, manager.go:58-60): one erased data
             shard, and e ~ U{1..10} erasures uniform over all 30 shards

Algorithmic bytes (L = 1202): encode k*L read + m*L written per block; decode (recover into an
output buffer) (k + e_d)*L per block with e_d >= 1 erased data shards, nothing for blocks whose
data shards all arrived. Prints one JSON line per config.

Beside each kernel: its traffic twin (include/fec_probe.h) at the kernel's own residency (the
same-shape figure, *_probe_TB/s) and the twin's best over residency and output placement
(*_probe_best_TB/s, bench.best_twin: the box's ceiling for the access shape), with the kernel's
fraction of each.
"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402  (best_twin, padded: the bench's ceiling search)

PAYLOAD, L, S = 1200, 1202, 1216


def timed(torch, fn, iters, bursts=5):
    """ms per launch: the median of `bursts` back-to-back bursts of `iters` launches (the first
    burst after a change of kernel runs up to 25 % slow for the 40-us RS(2,3) launches,
    tools/cb_probe.py)."""
    r = []
    for _ in range(bursts):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        r.append(s.elapsed_time(e) / iters)
    return sorted(r)[len(r) // 2]


def make_data(torch, B, k, g):
    data = torch.zeros((B, k, S), dtype=torch.uint8, device="cuda")
    for b0 in range(0, B, 1 << 16):
        b1 = min(B, b0 + (1 << 16))
        data[b0:b1, :, :PAYLOAD] = torch.randint(0, 256, (b1 - b0, k, PAYLOAD), generator=g, device="cuda",
                                                 dtype=torch.int16).to(torch.uint8)
    data[:, :, PAYLOAD] = PAYLOAD >> 8
    data[:, :, PAYLOAD + 1] = PAYLOAD & 0xFF
    return data


def twin_fields(torch, name, twin, nbytes, t_kernel, iters):
    """The twin at the kernel's residency and its best over residency and placement, with the
    kernel's fraction of each (t_kernel: ms per launch)."""
    same = round(nbytes / timed(torch, twin, iters) / 1e9, 3)
    best = bench.best_twin(torch, torch.cuda.current_stream(), twin, nbytes)
    if same > best["probe_best_TBps"]:   # the same-shape run (the kernel's own residency) won
        best.update(probe_best_TBps=same, probe_best_at="own residency")
    kern = nbytes / t_kernel / 1e9
    return {"%s_probe_TB/s" % name: same, "%s_frac_of_probe" % name: round(kern / same, 4),
            "%s_probe_best_TB/s" % name: best["probe_best_TBps"], "%s_probe_best_at" % name: best["probe_best_at"],
            "%s_frac_of_probe_best" % name: round(kern / best["probe_best_TBps"], 4)}


def run_rs(torch, fec, codec, k, m, B, multi, iters, seed):
    n = k + m
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    data = make_data(torch, B, k, g)
    parity = bench.padded(torch, (B, m, S), "cuda")
    if multi:
        # e ~ U{1..multi} erasures per block, a uniform subset of the n shards
        e = torch.randint(1, multi + 1, (B,), generator=g, device="cuda")
        keys = torch.rand((B, n), generator=g, device="cuda")
        rank = keys.argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
    else:
        which = torch.randint(0, k, (B,), generator=g, device="cuda")
        lost = torch.zeros((B, n), dtype=torch.bool, device="cuda")
        lost[torch.arange(B, device="cuda"), which] = True
    weights = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"),
                                       torch.arange(n, device="cuda"))
    masks = (((~lost).to(torch.int64) * weights).sum(dim=1)).to(torch.int32)
    e_d = lost[:, :k].sum(dim=1)
    slots = int(e_d.max().item())
    # multi-erasure configs: m output rows per block, as the rebuild traffic twin writes
    out = bench.padded(torch, (B, m if multi else max(slots, 1), S), "cuda")
    status = torch.zeros((B,), dtype=torch.int32, device="cuda")

    # raw C-ABI calls with the arguments precomputed: the shapes whose launches take tens of
    # microseconds (RS(2,3)) are otherwise timed at the Python call rate, not the device's
    dp, pp, op, mp, sp = data.data_ptr(), parity.data_ptr(), out.data_ptr(), masks.data_ptr(), status.data_ptr()
    slots_ = out.shape[1]

    def enc():
        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)

    def dec():
        rc = codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S, mp, op, slots_ * S, slots_, sp)
        if rc:
            raise fec.FecError(rc, "recover")

    enc()
    dec()
    codec.sync()
    # full-size check: recovered slot r of block b == its r-th erased data shard
    ok = bool((status == e_d.to(torch.int32)).all().item())
    order = torch.where(lost[:, :k], torch.arange(k, device="cuda"), k).sort(dim=1).values
    for r in range(slots):
        rows = (e_d > r).nonzero().squeeze(1)
        if rows.numel():
            src = data[rows, order[rows, r], :L]
            ok = ok and bool(torch.equal(out[rows, r, :L], src))
    for _ in range(2):
        enc()
        dec()
    torch.cuda.synchronize()
    t_enc = timed(torch, enc, iters)
    t_dec = timed(torch, dec, iters)
    enc_bytes = B * n * L
    dec_bytes = int(((k + e_d) * (e_d > 0)).sum().item()) * L
    # traffic twins (include/fec_probe.h): the kernels' bytes and launch shape without the field
    # arithmetic, timed after the kernels (they overwrite parity and out): this box's ceiling
    probe = {}
    if (k, m) in ((2, 1), (8, 4), (16, 8), (20, 10)):
        def enc_twin(wpc=-1, off=0):
            codec.probe_encode_traffic_raw(k, m, L, B, dp, k * S, pp + off, m * S, S, wpc)
        if multi and (k, m) in ((16, 8), (20, 10)):
            def dec_twin(wpc=-1, off=0):
                codec.probe_rebuild_traffic_raw(k, m, L, B, dp, k * S, pp, m * S, S, mp, op + off, slots_ * S, wpc)
        else:
            def dec_twin(wpc=-1, off=0):
                codec.probe_recover_traffic_raw(k, m, L, B, dp, k * S, pp, m * S, S, mp, op + off, slots_ * S, wpc)
        probe.update(twin_fields(torch, "encode", enc_twin, enc_bytes, t_enc, iters))
        probe.update(twin_fields(torch, "decode", dec_twin, dec_bytes, t_dec, iters))
    return {"config": "RS(%d,%d)" % (k, n), "blocks": B,
            "erasures": ("U{1..%d} of %d shards" % (multi, n)) if multi else "1 data shard",
            "mean_data_erasures": round(float(e_d.float().mean().item()), 3),
            "encode_ms": round(t_enc, 4), "decode_ms": round(t_dec, 4),
            "encode_TB/s": round(enc_bytes / t_enc / 1e9, 3), "decode_TB/s": round(dec_bytes / t_dec / 1e9, 3),
            "payload_GiB/s": round(B * k * PAYLOAD / 2**30 / ((t_enc + t_dec) / 1e3), 1),
            "step_frac": round((enc_bytes + dec_bytes) / ((t_enc + t_dec) / 1e3) / 8e12, 4),
            "check": ok, **probe}


def run_xor(torch, fec, codec, k, B, iters, seed):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    sh = torch.zeros((B, k + 1, S), dtype=torch.uint8, device="cuda")
    sh[:, :k] = make_data(torch, B, k, g)
    which = torch.randint(0, k, (B,), generator=g, device="cuda")
    masks = (((1 << (k + 1)) - 1) - torch.bitwise_left_shift(torch.ones_like(which), which)).to(torch.int32)
    ref = None

    shp, mp = sh.data_ptr(), masks.data_ptr()
    n = k + 1

    def enc():
        rc = fec.lib.fec_xor_encode_batch(codec.handle, k, L, B, shp, n * S, shp + k * S, n * S, S, fec.FEC_DEVICE)
        if rc:
            raise fec.FecError(rc, "xor encode")

    def dec():
        rc = fec.lib.fec_xor_reconstruct_batch(codec.handle, k, L, B, shp, n * S, shp + k * S, n * S, S, mp, None,
                                               fec.FEC_DEVICE)
        if rc:
            raise fec.FecError(rc, "xor reconstruct")

    enc()
    codec.sync()
    ref = sh[:, :k, :L].clone()
    sh[torch.arange(B, device="cuda"), which] = 0
    dec()
    codec.sync()
    ok = bool(torch.equal(sh[:, :k, :L], ref))
    del ref
    t_enc = timed(torch, enc, iters)
    t_dec = timed(torch, dec, iters)
    enc_bytes = B * (k + 1) * L
    dec_bytes = B * (k + 1) * L
    probe = {}
    if k == 2:
        # the RS(2,3) twins over the interleaved XOR layout: k reads + 1 write per block either way
        # (the decode twin writes the rebuilt shard to a separate buffer, as many bytes; the encode
        # twin writes the parity slots in place, so it is not moved)
        out = bench.padded(torch, (B, 1, S), "cuda")

        def enc_twin(wpc=-1, off=0):
            codec.probe_encode_traffic_raw(k, 1, L, B, shp, n * S, shp + k * S, n * S, S, wpc)

        def dec_twin(wpc=-1, off=0):
            codec.probe_recover_traffic_raw(k, 1, L, B, shp, n * S, shp + k * S, n * S, S, mp, out.data_ptr() + off,
                                            S, wpc)
        probe.update(twin_fields(torch, "encode", enc_twin, enc_bytes, t_enc, iters))
        probe.update(twin_fields(torch, "decode", dec_twin, dec_bytes, t_dec, iters))
    return {"config": "XOR(%d,1)" % k, "blocks": B, "erasures": "1 data shard",
            "encode_ms": round(t_enc, 4), "decode_ms": round(t_dec, 4),
            "encode_TB/s": round(enc_bytes / t_enc / 1e9, 3), "decode_TB/s": round(dec_bytes / t_dec / 1e9, 3),
            "payload_GiB/s": round(B * k * PAYLOAD / 2**30 / ((t_enc + t_dec) / 1e3), 1),
            "step_frac": round((enc_bytes + dec_bytes) / ((t_enc + t_dec) / 1e3) / 8e12, 4),
            "check": ok, **probe}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    ap.add_argument("--tune", default="", help="knob=value,... applied with Codec.set_tuning")
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    codec = fec.Codec(0).use_torch_stream()
    if args.tune:
        codec.set_tuning(**{kv.split("=")[0]: int(kv.split("=")[1]) for kv in args.tune.split(",")})
    cases = [("rs23", lambda: run_rs(torch, fec, codec, 2, 1, 65536, 0, max(args.iters, 100), 0x0FEC)),
             ("rs812", lambda: run_rs(torch, fec, codec, 8, 4, 1 << 20, 0, args.iters, 0x0FEC)),
             ("rs1624", lambda: run_rs(torch, fec, codec, 16, 8, 1 << 19, 8, args.iters, 0x0FEC)),
             ("xor21", lambda: run_xor(torch, fec, codec, 2, 1 << 20, args.iters, 0x0FEC)),
             # the reference's own factory code (manager.go:58-60), not a BASELINE config
             ("rs2030", lambda: run_rs(torch, fec, codec, 20, 10, 1 << 19, 0, args.iters, 0x0FEC)),
             ("rs2030m", lambda: run_rs(torch, fec, codec, 20, 10, 1 << 19, 10, args.iters, 0x0FEC))]
    for name, fn in cases:
        if args.only and name not in args.only.split(","):
            continue
        print(json.dumps(fn()), flush=True)
        torch.cuda.empty_cache()
    codec.close()


if __name__ == "__main__":
    main()
