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


if __name__ == "__main__":
    main()
