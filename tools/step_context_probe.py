#!/usr/bin/env python3
"""Diagnostics: does the headline encode run slower inside bench.py's step than alone?
Round 4's encode A/Bs (profiles/r04/enc_*_r04*.log) timed RS(8,12) encode back-to-back at
6.4-6.5 TB/s; the bench step (encode, then decode, alternating) sees 6.1. This times, in one process and interleaved over rounds, on the
bench's own buffers (bench.RankBatch / RankStep):
  enc x5       encode launches back-to-back
  dec x5       decode launches back-to-back
  step enc/dec encode and decode alternating, each bracketed by events (the bench's loop)
  enc, gap     each encode after a device-idle gap (host sync between launches)
usage: step_context_probe.py [rounds]"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    bench = importlib.import_module("bench")
    fec = importlib.import_module("0xfec_amd")
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    k, m, B = 8, 4, 1 << 20
    codec = fec.Codec(0)
    codec.prepare(k, m)
    codec.use_torch_stream()
    stream = torch.cuda.current_stream()
    batch = bench.RankBatch(torch, codec, torch.device("cuda", 0), B, k, m, 0x0FEC, 0)
    st = bench.RankStep(fec, codec, batch)
    enc_bytes = B * (k + m) * bench.SHARD_LEN
    dec_bytes = B * (k + 1) * bench.SHARD_LEN
    for _ in range(5):
        st.encode()
        st.decode()
    torch.cuda.synchronize()

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def burst(fn, n=5):
        a, b = ev(), ev()
        a.record(stream)
        for _ in range(n):
            fn()
        b.record(stream)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / n

    def step(n=5):
        es = [(ev(), ev(), ev()) for _ in range(n)]
        for e in es:
            e[0].record(stream)
            st.encode()
            e[1].record(stream)
            st.decode()
            e[2].record(stream)
        torch.cuda.synchronize()
        return (sum(e[0].elapsed_time(e[1]) for e in es) / n, sum(e[1].elapsed_time(e[2]) for e in es) / n)

    def gap(n=5):
        t = 0.0
        for _ in range(n):
            torch.cuda.synchronize()
            t += burst(st.encode, 1)
        return t / n

    res = {"enc x5": [], "dec x5": [], "step enc": [], "step dec": [], "enc, gap": []}
    for _ in range(rounds):
        res["enc x5"].append(burst(st.encode))
        res["dec x5"].append(burst(st.decode))
        e, d = step()
        res["step enc"].append(e)
        res["step dec"].append(d)
        res["enc, gap"].append(gap())
    out = {}
    for n, v in res.items():
        med = sorted(v)[len(v) // 2]
        by = dec_bytes if "dec" in n else enc_bytes
        out[n] = {"median_ms": round(med, 4), "TB/s": round(by / med / 1e9, 3), "min_ms": round(min(v), 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
