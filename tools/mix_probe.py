#!/usr/bin/env python3
"""Diagnostics: mixed read/write HBM rates vs output offset, XCD mapping, occupancy, items per
lane (tools/mix_probe.hip). Prints one JSON object; rates are bytes moved / time in GB/s.

usage: mix_probe.py [sweep1|sweep2|sweep3|persist|ipl|pol|lpol] [--rebuild] [--build-only]"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmix_probe.so")


def main():
    if not os.path.exists(SO) or "--rebuild" in sys.argv:
        subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-o", SO,
                               os.path.join(HERE, "mix_probe.hip")])
    if "--build-only" in sys.argv:
        return
    import torch
    lib = ctypes.CDLL(SO)
    vp, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    lib.mix_probe.argtypes = [vp, vp, sz, sz, sz, u, u, i, i, i, i, sz, vp]
    lib.mix_persist_probe.argtypes = [vp, vp, sz, sz, sz, u, u, i, i, i, i, sz, vp, vp]
    st = torch.cuda.current_stream().cuda_stream
    arena = torch.empty(24 << 30, dtype=torch.uint8, device="cuda")
    base = (arena.data_ptr() + (1 << 21) - 1) & ~((1 << 21) - 1)
    ss, cps = 1216, 76

    def run(nin, nout, B, in_bs, out_bs, off, ipl=1, swz=0, pad=0, iters=6):
        src = base
        dst = base + B * in_bs + off
        fn = lambda: lib.mix_probe(src, dst, in_bs, out_bs, ss, cps, B, nin, nout, ipl, swz, pad, st)
        if fn() != 0:
            return None
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        sec = s.elapsed_time(e) / iters / 1e3
        return round(B * cps * 16 * (nin + nout) / sec / 1e9, 1)

    res = {}
    mode = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else "sweep1"
    sys.stdout.write("probe start %s\n" % mode)
    sys.stdout.flush()

    def flush():
        sys.stdout.write(json.dumps(res) + "\n")
        sys.stdout.flush()

    if mode == "sweep1":
        Bc = 4 << 20                      # copy: 4M x 1216 B = 5.1 GB each way
        for off in (0, 256, 4096, 65536, (2 << 20) + 192, (33 << 20) + 4160):
            res["copy off%d" % off] = run(1, 1, Bc, ss, ss, off)
        for ipl in (2, 4):
            res["copy ipl%d" % ipl] = run(1, 1, Bc, ss, ss, 0, ipl=ipl)
        res["copy swz"] = run(1, 1, Bc, ss, ss, 0, swz=1)
        for pad in (32 * 1024 + 16, 54 * 1024, 80 * 1024):
            res["copy pad%d" % pad] = run(1, 1, Bc, ss, ss, 0, pad=pad)
        res["write"] = run(0, 1, Bc, ss, ss, 0)
        res["write ipl4"] = run(0, 1, Bc, ss, ss, 0, ipl=4)
        res["read8"] = run(8, 0, 1 << 20, 8 * ss, 4 * ss, 0)
        flush()
        B = 1 << 20
        for shape, nout, obs in (("enc", 4, 4 * ss), ("dec", 1, ss)):
            for off in (0, 4096, (1 << 20) + 4160):
                res["%s off%d" % (shape, off)] = run(8, nout, B, 8 * ss, obs, off)
            res["%s swz" % shape] = run(8, nout, B, 8 * ss, obs, 0, swz=1)
            res["%s ipl2" % shape] = run(8, nout, B, 8 * ss, obs, 0, ipl=2)
            res["%s ipl2 swz" % shape] = run(8, nout, B, 8 * ss, obs, 0, ipl=2, swz=1)
            for pad in (27 * 1024, 32 * 1024 + 16, 54 * 1024, 80 * 1024 + 16):
                res["%s pad%dK" % (shape, pad // 1024)] = run(8, nout, B, 8 * ss, obs, 0, pad=pad)
            flush()
        res["copy off0 again"] = run(1, 1, Bc, ss, ss, 0)
        res["enc off0 again"] = run(8, 4, B, 8 * ss, 4 * ss, 0)
    elif mode == "sweep2":
        # (a) read:write ratio at equal pattern, contiguous [B][nin] -> [B][nout]
        B = 1 << 20
        for nin, nout in ((1, 1), (2, 1), (4, 1), (8, 1), (2, 2), (4, 4), (8, 8), (8, 2), (4, 2), (8, 4),
                          (16, 8), (16, 3)):
            Bs = B if nin + nout <= 16 else B // 2
            res["r%d w%d" % (nin, nout)] = run(nin, nout, Bs, nin * ss, nout * ss, 0)
        flush()
        # (b) resident workgroups per CU (LDS pad: 160 KiB / pad), with and without XCD swizzle
        for nin, nout in ((8, 4), (8, 1), (1, 1)):
            for w, pad in ((1, 96 << 10), (2, 64 << 10), (3, 48 << 10), (4, 36 << 10), (5, 30 << 10), (6, 0)):
                for swz in (0, 1):
                    res["r%d w%d wg%d swz%d" % (nin, nout, w, swz)] = run(nin, nout, B, nin * ss, nout * ss, 0,
                                                                          swz=swz, pad=pad)
            flush()
    elif mode == "sweep3":
        # shard stride: 1216 (9.5 lines) vs 1280 (10 lines, line-aligned shards) vs 1024
        B = 1 << 20
        for nin, nout in ((8, 4), (8, 1), (8, 0)):
            for sst, c in ((1216, 76), (1280, 76), (1280, 80), (1024, 64), (1152, 72)):
                def run_ss(nin=nin, nout=nout, sst=sst, c=c, swz=0, pad=0):
                    fn = lambda: lib.mix_probe(base, base + B * nin * sst, nin * sst, max(1, nout) * sst, sst, c, B,
                                               nin, nout, 1, swz, pad, st)
                    fn()
                    torch.cuda.synchronize()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(6):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    sec = s.elapsed_time(e) / 6 / 1e3
                    return round(B * c * 16 * (nin + nout) / sec / 1e9, 1)
                res["r%d w%d ss%d cps%d" % (nin, nout, sst, c)] = run_ss()
                res["r%d w%d ss%d cps%d swz wg2" % (nin, nout, sst, c)] = run_ss(swz=1, pad=64 << 10)
            flush()
    elif mode == "ipl":
        # items per lane x resident workgroups per CU, XCD-contiguous order, interleaved rounds:
        # whether fewer waves with more loads each move the encode / decode shapes faster
        B = 1 << 20
        pads = {1: 96 << 10, 2: 64 << 10, 3: 48 << 10, 4: 36 << 10, 5: 30 << 10}
        acc = {}
        for rnd in range(3):
            for nin, nout in ((8, 4), (8, 1)):
                for ipl in (1, 2, 4):
                    for w, pad in pads.items():
                        acc.setdefault("r%d w%d ipl%d wg%d" % (nin, nout, ipl, w), []).append(
                            run(nin, nout, B, nin * ss, nout * ss, 0, ipl=ipl, swz=1, pad=pad))
        res.update({kk: sorted(v)[1] for kk, v in acc.items()})
    elif mode == "pol":
        # store cache policy x residency, interleaved rounds (round 6): decode shape (8 reads + 1
        # store), encode shape (8 + 4) and reads alone, bench layout
        lib.mix_pol_probe.argtypes = [vp, vp, sz, sz, sz, u, u, i, i, i, sz, vp]
        B = 1 << 20
        pads = {2: 64 << 10, 3: 48 << 10}
        acc = {}

        def runq(nin, nout, pol, pad, iters=6):
            fn = lambda: lib.mix_pol_probe(base, base + B * nin * ss, nin * ss, max(1, nout) * ss, ss, cps, B, nin,
                                           nout, pol, pad, st)
            if fn() != 0:
                return None
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            return round(B * cps * 16 * (nin + nout) / (s.elapsed_time(e) / iters / 1e3) / 1e9, 1)
        names = {0: "nt", 1: "plain", 2: "sc1", 3: "sc0sc1"}
        for rnd in range(3):
            for nin, nout, pols in ((8, 1, (0, 1, 2, 3)), (8, 4, (0, 1, 2, 3)), (8, 0, (0,))):
                for pol in pols:
                    for w, pad in pads.items():
                        acc.setdefault("r%d w%d %s wg%d" % (nin, nout, names[pol], w), []).append(
                            runq(nin, nout, pol, pad))
            res.update({kk: sorted(v)[len(v) // 2] for kk, v in acc.items()})
            flush()
    elif mode == "lpol":
        # load cache policy x store policy (round 6): encode shape (8 reads + 4 stores: nt / sc1 stores)
        # and decode shape (8 + 1: nt / nt sc1 stores), at 2 and 3 workgroups/CU, interleaved rounds
        lib.mix_lp_probe.argtypes = [vp, vp, sz, sz, sz, u, u, i, i, i, sz, vp]
        B = 1 << 20
        pads = {2: 64 << 10, 3: 48 << 10}
        lnames = {0: "nt", 1: "plain", 2: "sc1", 3: "ntsc1", 4: "sc0sc1"}
        snames = {0: "nt", 2: "sc1", 4: "ntsc1"}
        acc = {}

        def runl(nout, lp, sp, pad, iters=6):
            fn = lambda: lib.mix_lp_probe(base, base + B * 8 * ss, 8 * ss, nout * ss, ss, cps, B, nout, lp, sp, pad, st)
            if fn() != 0:
                return None
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            return round(B * cps * 16 * (8 + nout) / (s.elapsed_time(e) / iters / 1e3) / 1e9, 1)
        for rnd in range(3):
            for nout, sps in ((4, (0, 2)), (1, (0, 4))):
                for sp in sps:
                    for lp in range(5):
                        for w, pad in pads.items():
                            acc.setdefault("r8 w%d ld-%s st-%s wg%d" % (nout, lnames[lp], snames[sp], w), []).append(
                                runl(nout, lp, sp, pad))
            res.update({kk: sorted(v)[len(v) // 2] for kk, v in acc.items()})
            flush()
    elif mode == "persist":
        B = 1 << 20
        ctr = torch.zeros(1024, dtype=torch.int32, device="cuda")

        def runp(nin, nout, mode, wpc, iters=6):
            grid = 256 * wpc
            pad = {1: 96 << 10, 2: 64 << 10, 3: 48 << 10, 4: 36 << 10}[wpc]
            fn = lambda: lib.mix_persist_probe(base, base + B * nin * ss, nin * ss, nout * ss, ss, cps, B, nin, nout,
                                               mode, grid, pad, ctr.data_ptr(), st)
            if fn() != 0:
                return None
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            sec = s.elapsed_time(e) / iters / 1e3
            return round(B * cps * 16 * (nin + nout) / sec / 1e9, 1)
        for rnd in range(2):
            for nin, nout in ((8, 4), (8, 1)):
                for wpc in (2, 3):
                    res["r%d w%d flat swz wg%d #%d" % (nin, nout, wpc, rnd)] = run(
                        nin, nout, B, nin * ss, nout * ss, 0, swz=1, pad={2: 64 << 10, 3: 48 << 10}[wpc])
                    for md in (0, 1, 2):
                        res["r%d w%d persist%d wg%d #%d" % (nin, nout, md, wpc, rnd)] = runp(nin, nout, md, wpc)
            flush()
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
