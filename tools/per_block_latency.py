#!/usr/bin/env python3
"""Per-block cost of the per-block Go schemes (go/internal/fec/reed_solomon_hip.go, FEC_HIP=block)
for the reference's two codes: RS(20,30) (manager.go:58-59) and RS(8,12) (BASELINE config #3).
One block per call, as hipReedSolomonScheme makes it: fec_rs_encode_batch / a single-erasure
fec_rs_reconstruct_batch with FEC_HOST (pageable host buffers, staged through the library's
pinned memory, one H2D + kernel + D2H round trip, synchronous). The median of `reps` calls,
timed in Python around the ctypes call (ctypes adds ~1-2 us of the figure). One CPU core's
per-block time for the same codes is bench.py's cpu_baseline.single_core.

Prints one JSON line per code."""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

L = 1202


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=400)
    args = ap.parse_args()
    fec = importlib.import_module("0xfec_amd")
    codec = fec.Codec(0)
    for k, m in ((20, 10), (8, 4)):
        n = k + m
        rng = np.random.default_rng(k)
        codec.prepare(k, m)
        data = rng.integers(0, 256, (1, k, L), dtype=np.uint8)
        par = np.zeros((1, m, L), dtype=np.uint8)
        masks = np.array([((1 << n) - 1) & ~1], dtype=np.uint32)
        t_enc, t_dec = [], []
        for r in range(args.reps + 20):
            t0 = time.perf_counter()
            codec.rs_encode_raw(k, m, L, 1, data.ctypes.data, k * L, par.ctypes.data, m * L, L, fec.FEC_HOST)
            t1 = time.perf_counter()
            rc = codec.rs_reconstruct_raw(k, m, L, 1, data.ctypes.data, k * L, par.ctypes.data, m * L, L,
                                          masks.ctypes.data, None, fec.FEC_HOST)
            t2 = time.perf_counter()
            assert rc == 0
            if r >= 20:
                t_enc.append(t1 - t0)
                t_dec.append(t2 - t1)
        med = lambda v: sorted(v)[len(v) // 2] * 1e6
        print(json.dumps({"code": "RS(%d,%d)" % (k, n), "shard_len": L,
                          "gpu_per_block_us": {"encode": round(med(t_enc), 1), "reconstruct_1_erasure": round(med(t_dec), 1),
                                               "calls": args.reps, "form": "FEC_HOST, 1 block per call (hipReedSolomonScheme)"},
                          }), flush=True)
    codec.close()


if __name__ == "__main__":
    main()
