#!/usr/bin/env python3
"""Diagnostics for tests/test_gpu_codec.py::test_stream_switch_orders_shared_workspace: two
RS(16,24) multi-erasure batches reconstructed back to back on two torch streams through one
ctx (fec_ctx_set_stream between them). Prints, per mode and batch, how many blocks differ from
the originals. Modes: 'switch' (as the test), 'host_sync' (torch.cuda.synchronize between the
two launches), 'one_stream' (both on one stream)."""
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    fec = importlib.import_module("0xfec_amd")
    k, m, L, S = 16, 8, 1202, 1216
    n = k + m
    res = {}
    for mode in ("switch", "host_sync", "one_stream", "switch"):
        c = fec.Codec(0)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        if mode == "one_stream":
            streams[1] = streams[0]
        outs = []
        for i, B in enumerate((1 << 16, 1 << 15)):
            rng = np.random.default_rng(0x57 + i)
            sh = torch.zeros((B, n, S), dtype=torch.uint8, device="cuda")
            sh[:, :k, :L] = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).cuda()
            torch.cuda.synchronize()   # written on torch's stream: order it before the codec's
            c.set_stream(streams[i].cuda_stream)
            c.rs_encode(k, m, sh, shard_len=L)
            c.sync()
            e = rng.integers(0, m + 1, B)
            masks = np.empty(B, dtype=np.uint32)
            for b in range(B):
                lost = rng.choice(n, size=int(e[b]), replace=False)
                masks[b] = ((1 << n) - 1) & ~int(sum(1 << int(x) for x in lost))
            lostm = torch.from_numpy(((masks[:, None] >> np.arange(n)) & 1) == 0).cuda()
            outs.append((sh.clone(), sh, lostm, torch.from_numpy(masks.view(np.int32)).cuda()))
        for want, sh, lostm, dm in outs:
            sh[lostm] = 0x5A
        torch.cuda.synchronize()
        for i, (want, sh, lostm, dm) in enumerate(outs):
            c.set_stream(streams[i].cuda_stream)
            c.rs_reconstruct(k, m, sh, dm, shard_len=L)
            if mode == "host_sync":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        rc = c.lib_sync_rc()
        bad = []
        for want, sh, lostm, dm in outs:
            diff = (sh[:, :k, :L] != want[:, :k, :L]).any(dim=2).any(dim=1)
            bad.append(int(diff.sum().item()))
        res.setdefault(mode, []).append({"rc": rc, "bad_blocks_per_batch": bad})
        c.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
