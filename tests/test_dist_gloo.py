"""Multi-rank structure of the batch path on CPU (gloo, world_size 2): each rank owns a
contiguous block range (0xfec_amd/shard.py), codes it independently (the CPU oracle stands in
for the GPU kernels here; the GPU tests cover the kernels), and the only cross-rank traffic
is the timing reduction and a checksum gather. Rank 0 checks that the union of the ranks'
parity equals one process coding the whole batch, and the bench's aggregate formula."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, k, m, out_q):
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from oracle import oracle as orc
    shard = importlib.import_module("0xfec_amd.shard")
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method="tcp://127.0.0.1:%d" % port)
    lo, hi = shard.block_range(total, rank, world)
    L, S = 1202, 1216
    sh = np.zeros((hi - lo, k + m, S), dtype=np.uint8)
    sh[:, :k] = shard.synth_payload_blocks(0x0FEC, lo, hi, k, 1200, S)
    orc.rs_encode(k, m, sh, threads=1)
    parity = torch.from_numpy(np.ascontiguousarray(sh[:, k:, :L]).reshape(hi - lo, -1).astype(np.int64))
    digest = torch.zeros(total, dtype=torch.int64)
    digest[lo:hi] = (parity * torch.arange(1, parity.shape[1] + 1, dtype=torch.int64)).sum(dim=1)
    dist.all_reduce(digest, op=dist.ReduceOp.SUM)          # disjoint ranges: sum == gather
    t = torch.tensor([0.010 * (rank + 1)], dtype=torch.float64)   # per-rank step times
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    sizes = torch.zeros(world, dtype=torch.int64)
    sizes[rank] = hi - lo
    dist.all_reduce(sizes, op=dist.ReduceOp.SUM)
    if rank == 0:
        out_q.put((digest.numpy(), float(t.item()), sizes.tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total", [(2, 37), (2, 64)])
def test_sharded_batch_equals_single_process(world, total):
    import importlib
    from oracle import oracle as orc
    shard = importlib.import_module("0xfec_amd.shard")
    k, m = 8, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, k, m, q)) for r in range(world)]
    for p in procs:
        p.start()
    digest, tmax, sizes = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # single process reference
    sh = np.zeros((total, k + m, 1216), dtype=np.uint8)
    sh[:, :k] = shard.synth_payload_blocks(0x0FEC, 0, total, k, 1200, 1216)
    orc.rs_encode(k, m, sh, threads=1)
    par = sh[:, k:, :1202].reshape(total, -1).astype(np.int64)
    want = (par * np.arange(1, par.shape[1] + 1, dtype=np.int64)).sum(axis=1)
    assert np.array_equal(digest, want)
    assert sizes == [hi - lo for lo, hi in (shard.block_range(total, r, world) for r in range(world))]
    assert tmax == pytest.approx(0.010 * world)
    gib = shard.aggregate_gibps(sizes, k, 1200, tmax)
    assert gib == pytest.approx(total * k * 1200 / 2**30 / tmax)


def test_block_range_partitions():
    import importlib
    shard = importlib.import_module("0xfec_amd.shard")
    for total in (0, 1, 7, 8, 1 << 20, (1 << 23) + 3):
        for world in (1, 2, 3, 8):
            rs = [shard.block_range(total, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def test_synthetic_data_independent_of_split():
    import importlib
    shard = importlib.import_module("0xfec_amd.shard")
    whole = shard.synth_payload_blocks(7, 0, 10, 3, 1200, 1216)
    parts = np.concatenate([shard.synth_payload_blocks(7, lo, hi, 3, 1200, 1216) for lo, hi in ((0, 4), (4, 10))])
    assert np.array_equal(whole, parts)
    assert (whole[:, :, 1200] == 0x04).all() and (whole[:, :, 1201] == 0xB0).all()
    assert (whole[:, :, 1202:] == 0).all()
