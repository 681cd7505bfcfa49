#!/usr/bin/env python3
"""Diagnostics: HBM rate of the RS(8,12) encode and single-erasure decode access shapes with
the parity shards laid out [B][4][S] (the bench layout: a block's 4 parity shards together)
or [4][B][S] (parity row r of every block contiguous), pure traffic, interleaved A/B in one
process (tools/layout_probe.hip). Prints one JSON object: name -> [median, max] GB/s."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liblayout_probe.so")


def occupancy_lds(wpc):
    if wpc <= 0:
        return 0
    cu = 160 * 1024
    return ((cu // wpc + cu // (wpc + 1)) // 2) & ~255


def main():
    if not os.path.exists(SO) or "--rebuild" in sys.argv:
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                               os.path.join(HERE, "layout_probe.hip")])
    if "--build-only" in sys.argv:
        return
    import torch
    lib = ctypes.CDLL(SO)
    vp, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.layout_probe.argtypes = [i, vp, vp, vp, sz, sz, sz, sz, u, u, i, sz, vp]
    st = torch.cuda.current_stream().cuda_stream
    B, k, m, S, cps = 1 << 20, 8, 4, 1216, 76
    data = torch.empty(B * k * S, dtype=torch.uint8, device="cuda")
    par = torch.empty(B * m * S, dtype=torch.uint8, device="cuda")
    out = torch.empty(B * S, dtype=torch.uint8, device="cuda")
    layouts = {"[B][m][S]": (m * S, S), "[m][B][S]": (S, B * S)}
    cases = {}
    for lname, (pbs, pss) in layouts.items():
        for swz in (0, 1):
            for wpc in (0, 4):
                for shape in (0, 1):
                    name = "%s %s swz%d wpc%d" % ("enc" if shape == 0 else "dec", lname, swz, wpc)
                    cases[name] = (shape, pbs, pss, swz, occupancy_lds(wpc))

    def t(c, iters=5):
        shape, pbs, pss, swz, pad = c
        fn = lambda: lib.layout_probe(shape, data.data_ptr(), par.data_ptr(), out.data_ptr(), k * S, S, pbs, pss,
                                      cps, B, swz, pad, st)
        assert fn() == 0
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        sec = s.elapsed_time(e) / iters / 1e3
        return B * cps * 16 * ((k + m) if shape == 0 else (k + 1)) / sec / 1e9

    res = {n: [] for n in cases}
    for rnd in range(6):
        for n, c in cases.items():
            res[n].append(t(c))
        sys.stdout.write("round %d\n" % rnd)
        sys.stdout.flush()
    print(json.dumps({n: [round(sorted(v)[len(v) // 2], 1), round(max(v), 1)] for n, v in sorted(res.items())}))


if __name__ == "__main__":
    main()
