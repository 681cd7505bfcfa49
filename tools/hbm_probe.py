#!/usr/bin/env python3
"""Diagnostics: achievable HBM read / write / copy rates on this MI355X (16-B lanes)."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libhbm_probe.so")


def main():
    if not os.path.exists(SO):
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                               os.path.join(HERE, "hbm_probe.hip")])
    if len(sys.argv) > 1 and sys.argv[1] == "--build-only":
        return
    import torch
    lib = ctypes.CDLL(SO)
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    lib.probe_read.argtypes = [vp, sz, vp, i, i, i, vp]
    lib.probe_copy.argtypes = [vp, vp, sz, i, i, i, vp]
    lib.probe_write.argtypes = [vp, sz, i, i, vp]
    lib.probe_shards.argtypes = [vp, vp, sz, sz, ctypes.c_uint, ctypes.c_uint, i, i, i, i, vp, vp]
    lib.probe_store_policy.argtypes = [vp, vp, sz, sz, ctypes.c_uint, ctypes.c_uint, i, i, i, vp]
    if len(sys.argv) > 1 and sys.argv[1] == "--shards":
        return shards(lib, torch)
    if len(sys.argv) > 1 and sys.argv[1] == "--store-policy":
        return store_policy(lib, torch)
    nbytes = 8 << 30
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    out = torch.zeros(1 << 20, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def t(fn, iters=5):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    res = {}
    for grid in (1024, 2048, 4096, 16384):
        for unroll in (1, 4, 8):
            for nt in (0, 1):
                sec = t(lambda: lib.probe_read(a.data_ptr(), nbytes, out.data_ptr(), grid, unroll, nt, st))
                res["read g%d u%d nt%d" % (grid, unroll, nt)] = round(nbytes / sec / 1e9, 1)
    for grid in (1024, 2048, 4096, 16384):
        for unroll in (1, 4):
            for nt in (0, 1):
                sec = t(lambda: lib.probe_copy(a.data_ptr(), b.data_ptr(), nbytes, grid, unroll, nt, st))
                res["copy g%d u%d nt%d" % (grid, unroll, nt)] = round(2 * nbytes / sec / 1e9, 1)
    for grid in (1024, 4096, 16384):
        for nt in (0, 1):
            sec = t(lambda: lib.probe_write(b.data_ptr(), nbytes, grid, nt, st))
            res["write g%d nt%d" % (grid, nt)] = round(nbytes / sec / 1e9, 1)
    print(json.dumps(res, indent=1))


def store_policy(lib, torch):
    B, n, ss, cps = 1 << 20, 12, 1216, 76
    st = torch.cuda.current_stream().cuda_stream
    buf = torch.empty(B * n * ss, dtype=torch.uint8, device="cuda")
    obuf = torch.empty(B * n * ss, dtype=torch.uint8, device="cuda")
    base = buf.data_ptr()
    res = {}
    names = ["plain", "nt", "sc1", "sc0sc1", "sc1nt", "sc0sc1nt"]
    for rnd in range(2):
        for kin, nout, sep in ((8, 0, 0), (8, 1, 0), (8, 1, 1), (8, 4, 0), (8, 4, 1)):
            for pol in (0, 1, 4):
                ob = obuf.data_ptr() if sep else base + kin * ss
                fn = lambda: lib.probe_store_policy(base, ob, n * ss, ss, cps, B, kin, nout, pol, st)
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    fn()
                e.record()
                torch.cuda.synchronize()
                sec = s.elapsed_time(e) / 5 / 1e3
                res.setdefault("in%d out%d %s sep%d" % (kin, nout, names[pol], sep), []).append(
                    round(B * cps * 16 * (kin + nout) / sec / 1e9, 1))
    print(json.dumps(res, indent=1))


def shards(lib, torch):
    """Codec-shaped patterns: [B][12][ss] slots, kin loads + nout stores per 16-B item."""
    B = 1 << 20
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for ss in (1216, 1024, 1280):
        n = 12
        buf = torch.empty(B * n * ss, dtype=torch.uint8, device="cuda")
        sink = torch.zeros(16, dtype=torch.int32, device="cuda")
        cps = 1216 // 16 if ss >= 1216 else ss // 16
        base = buf.data_ptr()
        for kin, nout, in ((8, 0), (8, 1), (8, 4), (1, 1), (12, 0)):
            for nt in (0, 1):
                obase = base + kin * ss if nout else base
                fn = lambda: lib.probe_shards(base, obase, n * ss, ss, cps, B, kin, nout, nt, 0, sink.data_ptr(), st)
                fn()
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    fn()
                e.record()
                torch.cuda.synchronize()
                sec = s.elapsed_time(e) / 5 / 1e3
                by = B * cps * 16 * (kin + nout)
                res["ss%d in%d out%d nt%d" % (ss, kin, nout, nt)] = round(by / sec / 1e9, 1)
        del buf
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
