#!/usr/bin/env python3
"""Diagnostics: the RS(8,12) encode and its traffic twin (include/fec_probe.h) at several
residencies (knob enc_wpc: workgroups per CU, 0 uncapped), interleaved bursts in one process.
Says whether the encode's access shape moves more at another residency than the one the encode
runs at, i.e. whether a form of the encode with more work per lane at lower residency could beat
the ceiling the bench reports.

(Round 6 ran it with two measurement-only forms beside the encode, knobs enc_lite and enc_scal,
removed after: profiles/r06/twin_sweep_lite_r06n.log, twin_sweep_scal_r06o.log.)

usage: twin_sweep.py [blocks]   (2^20 default)"""
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, L, S = 8, 4, 1202, 1216
    pos = [x for x in sys.argv[1:] if not x.startswith("--")]
    B = int(pos[0]) if pos else 1 << 20
    codec = fec.Codec(0).use_torch_stream()
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    dp, pp = data.data_ptr(), par.data_ptr()
    nbytes = B * (k + m) * L

    def kern():
        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE)

    def twin():
        codec.probe_encode_traffic_raw(k, m, L, B, dp, k * S, pp, m * S, S)

    def t(fn, iters=5):
        fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    base = codec.set_tuning(enc_wpc=3)
    res = {}
    for _ in range(7):
        for w in (2, 3, 4, 5, 0):
            codec.set_tuning(enc_wpc=w)
            for name, fn in (("encode", kern), ("twin", twin)):
                res.setdefault("%s wpc%d" % (name, w), []).append(nbytes / t(fn) / 1e12)
    codec.set_tuning(**base)
    print(json.dumps({n: round(sorted(v)[len(v) // 2], 3) for n, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
