#!/usr/bin/env python3
"""Host-resident (PCIe-inclusive) FEC throughput on one MI355X.

The reference's path starts and ends in host memory (QUIC packet buffers: repair_queue.go,
packet_packer.go:980-1016, connection.go:1305-1376). This measures the codec with its inputs
and outputs in pinned host memory: chunks of blocks are copied H2D, coded on the device and
copied D2H, with copies and kernels of neighbouring chunks overlapped on two HIP streams.

    encode: H2D k data shards, fec_rs_encode_batch, D2H m parity shards
    decode: H2D k data shards (one erased) + parity shard 0, fec_rs_recover_batch,
            D2H the recovered shard

Reports payload GiB/s (k * 1200 bytes per block) and the PCIe byte rate each direction.
"""
import argparse
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=1 << 18)
    ap.add_argument("--chunk", type=int, default=1 << 14)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, B, C = args.k, args.m, args.blocks, args.chunk
    L, S = 1202, 1216
    dev = torch.device("cuda", 0)
    codec = fec.Codec(0)
    codec.prepare(k, m)
    data_h = torch.randint(0, 256, (B, k, S), dtype=torch.uint8).pin_memory()
    parity_h = torch.zeros((B, m, S), dtype=torch.uint8).pin_memory()
    rec_h = torch.zeros((B, 1, S), dtype=torch.uint8).pin_memory()
    erased = torch.randint(0, k, (B,))
    masks_h = ((1 << (k + m)) - 1 - (1 << erased)).to(torch.int32).pin_memory()
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    bufs = [dict(d=torch.empty((C, k, S), dtype=torch.uint8, device=dev),
                 p=torch.empty((C, m, S), dtype=torch.uint8, device=dev),
                 r=torch.empty((C, 1, S), dtype=torch.uint8, device=dev),
                 mk=torch.empty((C,), dtype=torch.int32, device=dev)) for _ in streams]

    def run_encode():
        for i, b0 in enumerate(range(0, B, C)):
            nb = min(C, B - b0)
            s, bf = streams[i % 2], bufs[i % 2]
            with torch.cuda.stream(s):
                bf["d"][:nb].copy_(data_h[b0:b0 + nb], non_blocking=True)
                codec.set_stream(s.cuda_stream)
                codec.rs_encode_raw(k, m, L, nb, bf["d"].data_ptr(), k * S, bf["p"].data_ptr(), m * S, S,
                                    fec.FEC_DEVICE)
                parity_h[b0:b0 + nb].copy_(bf["p"][:nb], non_blocking=True)

    def run_decode():
        for i, b0 in enumerate(range(0, B, C)):
            nb = min(C, B - b0)
            s, bf = streams[i % 2], bufs[i % 2]
            with torch.cuda.stream(s):
                bf["d"][:nb].copy_(data_h[b0:b0 + nb], non_blocking=True)
                bf["p"][:nb, :1].copy_(parity_h[b0:b0 + nb, :1], non_blocking=True)
                bf["mk"][:nb].copy_(masks_h[b0:b0 + nb], non_blocking=True)
                codec.set_stream(s.cuda_stream)
                rc = codec.rs_recover_raw(k, m, L, nb, bf["d"].data_ptr(), k * S, bf["p"].data_ptr(), m * S, S,
                                          bf["mk"].data_ptr(), bf["r"].data_ptr(), S, 1, None)
                assert rc == 0
                rec_h[b0:b0 + nb].copy_(bf["r"][:nb], non_blocking=True)

    res = {}
    for name, fn, up, down in (("encode", run_encode, k * S, m * S), ("decode", run_decode, (k + 1) * S, S)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.iters
        res[name] = {"payload_GiB/s": round(B * k * 1200 / 2**30 / dt, 2), "ms": round(dt * 1e3, 3),
                     "h2d_GB/s": round(B * up / dt / 1e9, 1), "d2h_GB/s": round(B * down / dt / 1e9, 1)}
    # check: recovered shards equal the erased originals
    ok = bool(torch.equal(rec_h[:, 0, :L], data_h[torch.arange(B), erased, :L]))
    t_both = res["encode"]["ms"] + res["decode"]["ms"]
    res["encode+decode_payload_GiB/s"] = round(B * k * 1200 / 2**30 / (t_both / 1e3), 2)
    res["recovered_ok"] = ok
    res["config"] = {"k": k, "m": m, "blocks": B, "chunk_blocks": C, "streams": 2, "host_memory": "pinned"}
    print(json.dumps(res))
    codec.close()


if __name__ == "__main__":
    main()
