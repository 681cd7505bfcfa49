#!/usr/bin/env python3
"""Diagnostics: pick the single-erasure recover launch form by interleaved A/B in one process
(plan kernel + wave rebuild vs the direct form, residency caps, XCD order), many rounds.
Every variant's output is checked against the default's first.

usage: dec_select.py [--k 8 --m 4 --blocks 1048576] [--rounds 8]"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--blocks", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tiers", action="store_true", help="A/B the two-tier rebuild (knob dec_tier) only")
    ap.add_argument("--multi", type=int, default=0,
                    help="e ~ U{1..multi} erasures uniform over all n shards (config_bench's RS(16,24) mix)")
    ap.add_argument("--only", default="", help="comma-separated substrings: keep the variants naming one (and the default)")
    args = ap.parse_args()
    import torch
    fec = importlib.import_module("0xfec_amd")
    B, k, m, L, S = args.blocks, args.k, args.m, 1202, 1216
    codec = fec.Codec(0).use_torch_stream()
    data = torch.randint(0, 256, (B, k, S), dtype=torch.uint8, device="cuda")
    par = torch.randint(0, 256, (B, m, S), dtype=torch.uint8, device="cuda")
    n = k + m
    if args.multi:
        e = torch.randint(1, args.multi + 1, (B,), device="cuda")
        rank = torch.rand((B, n), device="cuda").argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
        weights = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"),
                                           torch.arange(n, device="cuda"))
        masks = (((~lost).to(torch.int64) * weights).sum(dim=1)).to(torch.int32)
        slots = max(1, int(lost[:, :k].sum(dim=1).max().item()))
        e_d = lost[:, :k].sum(dim=1)
        byts_total = int(((k + e_d) * (e_d > 0)).sum().item()) * L
    else:
        erased = torch.randint(0, k, (B,), device="cuda")
        masks = ((1 << n) - 1 - (1 << erased)).to(torch.int32)
        slots = 1
        byts_total = B * (k + 1) * L
    out = torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda")
    status = torch.zeros((B,), dtype=torch.int32, device="cuda")
    dp, pp, op = data.data_ptr(), par.data_ptr(), out.data_ptr()
    # every knob any variant sets, at its default: tune(D) must undo each variant completely
    D = dict(dec_wave=1, dec_fused=0, dec_wpc=0, dec_swz=1, dec_ipl=0, dec_direct=1, dec_nt=3, dir_wpc=-1, dir_nt=-1,
             dec_fixk=4, dec_sorted=1, dec_pseg=0, dec_tier=0, dec_direct_big=0, dec_gate=0, dec_gate_pm=10, dec_win=0, dec_s64=0, dec_psort=1, dec_pv=3, dec_povl=0, dec_lpad=0, dec_rwin=4)
    variants = {"direct (default)": D,
                "direct, PermTab rows by vector load": dict(D, dec_direct=2),
                "direct noswz": dict(D, dec_swz=0),
                "plan + wave": dict(D, dec_direct=0)}
    for w in (0, 2, 3, 4, 6):
        for nt, nm in ((3, "nt"), (2, "plain loads")):
            variants["direct wpc%d, %s" % (w, nm)] = dict(D, dir_wpc=w, dir_nt=nt)
    variants["direct + status array"] = dict(D, _status=1)
    variants["direct, plain loads and stores"] = dict(D, dir_nt=0)
    if args.multi:   # the plan + wave path: residency, cache policy, compile-time k, plan form
        variants = {"default": D}
        variants["wave runtime k"] = dict(D, dec_fixk=0)
        variants["compile-time k, all k loads up front"] = dict(D, dec_fixk=1)
        variants["rolling window (fixk 2, round-2 default)"] = dict(D, dec_fixk=2)
        variants["rolling window + row-pipelined tables (fixk 3)"] = dict(D, dec_fixk=3)
        variants["table-copy rebuild (fixk 4)"] = dict(D, dec_fixk=4)
        for w in (4, 6, 8):
            variants["table-copy rebuild (fixk 4) window %d" % w] = dict(D, dec_fixk=4, dec_win=w)
            variants["table-copy rebuild (fixk 4) window %d, 64-bit split shifts" % w] = dict(D, dec_fixk=4, dec_win=w, dec_s64=1)
        for w in (2, 3):
            variants["table-copy rebuild (fixk 4) wpc%d" % w] = dict(D, dec_fixk=4, dec_wpc=w)
        for ps in (0, 2, 4):
            variants["table-copy rebuild (fixk 4), plans sorted over %d blocks" % (64 * ps)] = dict(D, dec_fixk=4, dec_psort=ps)
        variants["plan form 1 (round 3)"] = dict(D, dec_pv=1)
        variants["plan form 2 (runtime code)"] = dict(D, dec_pv=2)
        variants["plan form 3 paired segments"] = dict(D, dec_pv=4)
        for w in (1, 2, 4, 8):
            variants["plan rank-first window %d" % (64 * w)] = dict(D, dec_pv=5, dec_rwin=w)
        variants["padded rebuild slice (lpad)"] = dict(D, dec_lpad=1)
        variants["padded rebuild slice (lpad), wpc 3"] = dict(D, dec_lpad=1, dec_wpc=3)
        for ov in (2, 4, 8):
            variants["plan overlap %d sub-batches" % ov] = dict(D, dec_povl=ov)
        for w in (3, 4):
            variants["rolling window wpc%d" % w] = dict(D, dec_wpc=w)
        for w in (2, 3):
            variants["K=16 wpc%d" % w] = dict(D, dec_wpc=w)
        variants["unsorted plans"] = dict(D, dec_sorted=0)
        for ps in (1, 2, 4, 8, 16):
            variants["plan segs %d" % ps] = dict(D, dec_pseg=ps)
        variants["default + status array"] = dict(D, _status=1)
    if args.tiers:
        variants = {"default": D}
        for rt in (2, 4):
            variants["tier %d" % rt] = dict(D, dec_tier=rt)
        if k in (16, 20):
            for w in (0, 4, 3):
                variants["direct_big wpc%d" % w] = dict(D, dec_direct_big=1, dir_wpc=w)
                variants["gated wpc%d" % w] = dict(D, dec_direct_big=1, dec_gate=1, dir_wpc=w)
    if args.only:
        keys = [x for x in args.only.split(",") if x]
        variants = {n: kv for n, kv in variants.items() if kv is D or any(x in n for x in keys)}
    base = codec.set_tuning(**D)
    use_status = [False]

    def run():
        codec.rs_recover_raw(k, m, L, B, dp, k * S, pp, m * S, S, masks.data_ptr(), op, slots * S, slots,
                             status.data_ptr() if use_status[0] else None)

    def t(iters):
        run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            run()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / iters / 1e3

    run()
    torch.cuda.synchronize()
    ref = out.clone()
    def tune(kv):
        use_status[0] = bool(kv.get("_status"))
        codec.set_tuning(**{x: y for x, y in kv.items() if not x.startswith("_")})

    for n, kv in variants.items():
        tune(kv)
        out.zero_()
        run()
        torch.cuda.synchronize()
        assert torch.equal(out, ref), n
        tune(D)
    res = {n: [] for n in variants}
    for _ in range(args.rounds):
        for n, kv in variants.items():
            tune(kv)
            res[n].append(t(args.iters))
            tune(D)
    byts = byts_total
    print(json.dumps({"shape": "RS(%d,%d) x %d%s" % (k, k + m, B, " e~U{1..%d}" % args.multi if args.multi else ""),
                      "median_us_TBps_best": {n: [round(sorted(v)[len(v) // 2] * 1e6, 1),
                                                  round(byts / sorted(v)[len(v) // 2] / 1e12, 3),
                                                  round(byts / min(v) / 1e12, 3)] for n, v in res.items()}}))


if __name__ == "__main__":
    main()
