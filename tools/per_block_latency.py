#!/usr/bin/env python3
"""Per-block cost of the per-block Go schemes (go/internal/fec/reed_solomon_hip.go, FEC_HIP=block)
against one CPU core doing the same block with klauspost's SIMD method (oracle/fec_simd.c, the
CPU baseline's restatement), for the reference's two codes: RS(20,30) (manager.go:58-59) and
XOR-free RS(8,12) (BASELINE config #3).

GPU: one block per call, as hipReedSolomonScheme makes it: fec_rs_encode_batch / a single-erasure
fec_rs_reconstruct_batch with FEC_HOST (pageable host buffers, staged through the library's
pinned memory, one H2D + kernel + D2H round trip, synchronous). The median of `reps` calls,
timed in Python around the ctypes call (ctypes adds ~1-2 us of the figure).
CPU: the same encode + reconstruct on one thread over `cpu_blocks` blocks, divided by the block
count (per-block throughput cost of one core; the fastest ISA the host has).

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
    ap.add_argument("--cpu-blocks", type=int, default=4096)
    args = ap.parse_args()
    fec = importlib.import_module("0xfec_amd")
    from oracle import oracle as orc
    orc.build()
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
        # one CPU core, klauspost's SIMD method, amortised over cpu_blocks blocks
        B = args.cpu_blocks
        sh = np.zeros((B, n, L), dtype=np.uint8)
        sh[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
        cmask = np.full(B, ((1 << n) - 1) & ~1, dtype=np.uint32)
        isas = [i for i in (orc.ISA_AVX2, orc.ISA_GFNI_AVX2, orc.ISA_GFNI_AVX512) if orc.isa_supported(i)]
        best = None
        for isa in isas:
            orc.rs_encode_simd(k, m, sh, isa, threads=1)
            te = min(_time(lambda: orc.rs_encode_simd(k, m, sh, isa, threads=1)) for _ in range(3))
            td = min(_time(lambda: orc.rs_reconstruct_simd(k, m, sh, cmask, isa, threads=1)) for _ in range(3))
            if best is None or te + td < best[1] + best[2]:
                best = (orc.isa_name(isa), te, td)
        med = lambda v: sorted(v)[len(v) // 2] * 1e6
        print(json.dumps({"code": "RS(%d,%d)" % (k, n), "shard_len": L,
                          "gpu_per_block_us": {"encode": round(med(t_enc), 1), "reconstruct_1_erasure": round(med(t_dec), 1),
                                               "calls": args.reps, "form": "FEC_HOST, 1 block per call (hipReedSolomonScheme)"},
                          "cpu_one_core_per_block_us": {"encode": round(best[1] / B * 1e6, 2),
                                                        "reconstruct_1_erasure": round(best[2] / B * 1e6, 2),
                                                        "isa": best[0], "blocks": B}}), flush=True)
    codec.close()


def _time(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


if __name__ == "__main__":
    main()
