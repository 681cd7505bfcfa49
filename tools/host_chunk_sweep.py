#!/usr/bin/env python3
"""Chunk size and parity-plane policy of the host-resident pipeline (fec_capi.cpp HostPipe),
measured with bench.py's own host_resident() step (RS(8,12) encode + single-erasure reconstruct,
packed pinned and pageable host buffers).

    python tools/host_chunk_sweep.py [--blocks 131072] [--threads 4,8,12,16 [--reps 3]]

One JSON line per setting of knob host_chunk (blocks per chunk; 0 = the library's default: up to
128 MiB of staged shards, a mid-sized call split over the three staging sets), or of host_threads
with --threads. (Round 4 also swept host_gather, the parity-plane policy; round 5 fixed it to the
measured rule, sparse planes pulled by the device and dense ones by 2D DMA, and removed the knob.)"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=1 << 17)
    ap.add_argument("--chunks", default="0,2048,4096,8192,16384,32768")
    ap.add_argument("--threads", default="", help="sweep knob host_threads instead (comma list), interleaved")
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch
    bench = importlib.import_module("bench")
    fec = importlib.import_module("0xfec_amd")
    codec = fec.Codec(0)
    codec.prepare(8, 4)
    if args.threads:
        res = {}
        for _ in range(args.reps):
            for t in [int(x) for x in args.threads.split(",")]:
                old = codec.set_tuning(host_threads=t)
                r = bench.host_resident(torch, fec, codec, 8, 4, args.blocks, 0x0FEC)
                codec.set_tuning(**old)
                key = "threads%d" % t
                res.setdefault(key, []).append((r["pageable"]["value"], r["pinned"]["value"]))
                print(json.dumps({"host_threads": t, "pageable": r["pageable"]["value"],
                                  "pinned": r["pinned"]["value"]}), flush=True)
        print(json.dumps({"median_pageable_GiBps": {t: sorted(v[0] for v in vs)[len(vs) // 2] for t, vs in res.items()},
                          "median_pinned_GiBps": {t: sorted(v[1] for v in vs)[len(vs) // 2] for t, vs in res.items()}}))
        codec.close()
        return
    for chunk in [int(c) for c in args.chunks.split(",")]:
        old = codec.set_tuning(host_chunk=chunk)
        r = bench.host_resident(torch, fec, codec, 8, 4, args.blocks, 0x0FEC)
        codec.set_tuning(**old)
        print(json.dumps({"host_chunk": chunk, "link_bound_GiBps": r["link_bound_GiBps"],
                          "pinned": r["pinned"], "pageable": r["pageable"]}), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
