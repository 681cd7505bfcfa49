#!/usr/bin/env python3
"""Diagnostics: the codec kernels beside pure-traffic probes of the same access shape, on the
same buffers, interleaved in one process (tools/mix_probe.hip). Rates are algorithmic bytes /
time (codec) or bytes moved / time (probe), GB/s."""
import ctypes
import importlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    so = os.path.join(HERE, "libmix_probe.so")
    if not os.path.exists(so):
        subprocess.check_call([sys.executable, os.path.join(HERE, "mix_probe.py"), "--build-only"])
    import torch
    fec = importlib.import_module("0xfec_amd")
    probe = ctypes.CDLL(so)
    vp, sz, i, u = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint
    probe.mix_probe.argtypes = [vp, vp, sz, sz, sz, u, u, i, i, i, i, sz, vp]
    probe.mix_persist_probe.argtypes = [vp, vp, sz, sz, sz, u, u, i, i, i, i, sz, vp, vp]
    B, k, m, L, S = 1 << 20, 8, 4, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    st = torch.cuda.current_stream().cuda_stream
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    erased = torch.randint(0, k, (B,), device="cuda")
    masks = ((1 << (k + m)) - 1 - (1 << erased)).to(torch.int32)
    ctr = torch.zeros(1024, dtype=torch.int32, device="cuda")
    cps = 76

    def t(fn, iters=6):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    dp, pp, op = data.data_ptr(), par.data_ptr(), out.data_ptr()
    cases = {
        "codec encode (queue kernel)": (lambda: codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE),
                                        B * (k + m) * L),
        "codec encode, no field math (diag)": (lambda: (codec.set_tuning(enc_diag=1),
                                                        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S,
                                                                            fec.FEC_DEVICE),
                                                        codec.set_tuning(enc_diag=0)), B * (k + m) * L),
        "codec encode qwpc3": (lambda: (codec.set_tuning(enc_qwpc=3),
                                        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE),
                                        codec.set_tuning(enc_qwpc=2)), B * (k + m) * L),
        "codec encode qwpc4": (lambda: (codec.set_tuning(enc_qwpc=4),
                                        codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE),
                                        codec.set_tuning(enc_qwpc=2)), B * (k + m) * L),
        "codec encode flat fixed wpc4": (lambda: (codec.set_tuning(enc_queue=0, enc_wpc=4),
                                                  codec.rs_encode_raw(k, m, L, B, dp, k * S, pp, m * S, S, fec.FEC_DEVICE),
                                                  codec.set_tuning(enc_queue=1, enc_wpc=3)), B * (k + m) * L),
        "probe 8r4w flat swz wg2": (lambda: probe.mix_probe(dp, pp, k * S, m * S, S, cps, B, 8, 4, 1, 1, 64 << 10, st),
                                    B * cps * 16 * 12),
        "probe 8r4w ticket-queue wg2": (lambda: probe.mix_persist_probe(dp, pp, k * S, m * S, S, cps, B, 8, 4, 1, 512,
                                                                        64 << 10, ctr.data_ptr(), st), B * cps * 16 * 12),
        "codec recover (plan + wave kernel)": (lambda: codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S,
                                                                            masks.data_ptr(), op, S, 1, None),
                                               B * (k + 1) * L),
        "probe 8r1w flat": (lambda: probe.mix_probe(dp, op, k * S, S, S, cps, B, 8, 1, 1, 0, 0, st), B * cps * 16 * 9),
        "probe 8r1w flat swz wg3": (lambda: probe.mix_probe(dp, op, k * S, S, S, cps, B, 8, 1, 1, 1, 48 << 10, st),
                                    B * cps * 16 * 9),
        "probe 8r1w ticket-queue wg3": (lambda: probe.mix_persist_probe(dp, op, k * S, S, S, cps, B, 8, 1, 1, 768,
                                                                        48 << 10, ctr.data_ptr(), st), B * cps * 16 * 9),
    }
    res = {n: [] for n in cases}
    for _ in range(4):
        for n, (fn, by) in cases.items():
            res[n].append(by / t(fn) / 1e9)
    print(json.dumps({n: round(sorted(v)[len(v) // 2], 1) for n, v in res.items()}, indent=1))


if __name__ == "__main__":
    main()
