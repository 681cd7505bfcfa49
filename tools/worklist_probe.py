#!/usr/bin/env python3
"""Diagnostics: many small RS(8,12) recover batches (FEC_DEVICE, mixed shard lengths and 0..m
erasures, out_slots = the batch's largest data-erasure count), each recovered shard checked against
the data the batch was encoded from (parity by the library's own encode; parity against the oracle
is the tests' job), with the direct decode's multi-erasure worklist state read back after every
call."""
import ctypes
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    fec = importlib.import_module("0xfec_amd")
    codec = fec.Codec(0)
    fn = fec.lib.fec__worklist_state
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    st2 = (ctypes.c_uint32 * 2)()
    rng = np.random.default_rng(3)
    k, m = 8, 4
    n = k + m
    bad = 0
    for it in range(300):
        B = int(rng.integers(1, 4))
        L = int(rng.choice([3, 19, 602, 1202, 1436]))
        S = (L + 15) // 16 * 16
        full = np.zeros((B, n, L), dtype=np.uint8)
        full[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
        pad = np.zeros((B, n, S), dtype=np.uint8)
        pad[:, :, :L] = full
        enc = torch.from_numpy(pad).cuda()
        rc = codec.rs_encode_raw(k, m, L, B, enc.data_ptr(), n * S, enc.data_ptr() + k * S, n * S, S, fec.FEC_DEVICE)
        codec.sync()
        assert rc == 0
        full = np.ascontiguousarray(enc.cpu().numpy()[:, :, :L])
        masks = np.empty(B, dtype=np.uint32)
        for b in range(B):
            e = int(rng.integers(0, m + 1))
            lost = rng.choice(n, size=e, replace=False)
            masks[b] = ((1 << n) - 1) & ~int(sum(1 << int(i) for i in lost))
        ed = [k - bin(int(x) & ((1 << k) - 1)).count("1") for x in masks]
        slots = max(1, max(ed))
        sh = np.zeros((B, n, S), dtype=np.uint8)
        sh[:, :, :L] = full
        for b in range(B):
            for i in range(n):
                if not (masks[b] >> i) & 1:
                    sh[b, i] = 0xEE
        d = torch.from_numpy(sh).cuda()
        out = torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda")
        mk = torch.from_numpy(masks.view(np.int32)).cuda()
        status = torch.zeros(B, dtype=torch.int32, device="cuda")
        rc = codec.rs_recover_raw(k, m, L, B, d.data_ptr(), n * S, d.data_ptr() + k * S, n * S, S, mk.data_ptr(),
                                  out.data_ptr(), slots * S, slots, status.data_ptr())
        rs = codec.lib_sync_rc()
        fn(codec.handle, st2)
        o = out.cpu().numpy()
        stt = status.cpu().numpy()
        for b in range(B):
            if stt[b] < 0:
                continue
            lostd = [i for i in range(k) if not (masks[b] >> i) & 1]
            for r, i in enumerate(lostd):
                if not np.array_equal(o[b, r, :L], full[b, i]):
                    bad += 1
                    print("MISMATCH it=%d B=%d L=%d slots=%d block=%d e_d=%d status=%d rc=%d sync=%d wl=%s" % (
                        it, B, L, slots, b, len(lostd), stt[b], rc, rs, list(st2)), flush=True)
                    break
        if st2[0] or st2[1]:
            print("STALE worklist after it=%d: %s (B=%d L=%d slots=%d)" % (it, list(st2), B, L, slots), flush=True)
            break
    print("done, mismatches:", bad)


if __name__ == "__main__":
    main()
