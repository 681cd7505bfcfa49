"""GPU parity of the sender-side batching layer: the repair frames a connection's RepairQueue
receives from the batched path equal, in order and byte for byte, the frames the per-block
path (Manager.AddSourceSymbolFrame -> repairSymbols, manager.go:123-158) returns for the same
source symbols — across batch boundaries, double-buffered batches, mixed symbol lengths and
several connections sharing one encoder."""
import importlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B(fec):
    return importlib.import_module("0xfec_amd.batch")


@pytest.fixture(scope="module")
def S(fec):
    return importlib.import_module("0xfec_amd.scheme")


def _streams(rng, nconn, nblocks, k, lens):
    """Per connection: nblocks*k source payloads with lengths drawn from `lens`."""
    out = []
    for _ in range(nconn):
        pl = []
        for _ in range(nblocks * k):
            n = int(rng.choice(lens))
            pl.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        out.append(pl)
    return out


@pytest.mark.parametrize("scheme,k,m,max_blocks,lens", [
    ("rs", 20, 10, 4, [1200]),                       # the reference's RS factory code
    ("rs", 8, 4, 5, [1, 17, 600, 1200, 1434]),       # mixed lengths: slot-overflow flushes
    ("rs", 2, 1, 64, [1200, 1434]),
    ("xor", 2, 1, 3, [1, 100, 1200, 1434]),          # the reference's XOR factory code
])
def test_batched_frames_equal_per_block_frames(B, S, scheme, k, m, max_blocks, lens):
    rng = np.random.default_rng(k * 100 + max_blocks)
    sid = S.XOR_FEC_SCHEME if scheme == "xor" else S.REED_SOLOMON_FEC_SCHEME
    nconn, nblocks = 3, 7
    streams = _streams(rng, nconn, nblocks, k, lens)
    # per-block path
    want = []
    for pl in streams:
        mgr, err = S.new_manager(sid, k, m)
        assert err is None
        frames = []
        for ssid, p in enumerate(pl):
            fr, err = mgr.add_source_symbol_frame(ssid, p)
            assert err is None
            frames += fr or []
        want.append(frames)
    # batched path: one encoder for all connections, symbols interleaved across connections
    enc, err = B.BatchEncoder.new(sid, k, m, max_blocks=max_blocks)
    assert err is None
    mgrs = [S.new_manager(sid, k, m)[0] for _ in range(nconn)]
    queues = [B.RepairQueue(max_len=nblocks * m) for _ in range(nconn)]
    for ssid in range(nblocks * k):
        for c in range(nconn):
            assert mgrs[c].add_source_symbol_frame_batched(ssid, streams[c][ssid], enc, queues[c]) is None
        if ssid % 9 == 4:
            n, err = enc.poll()
            assert err is None
    n, err = enc.drain()
    assert err is None
    assert enc.staged == 0 and enc.in_flight == 0
    for c in range(nconn):
        cap = queues[c].peek_cap()
        assert cap == (len(want[c][0][2]) if scheme == "xor" else S.MAX_PACKET_BUFFER_SIZE)
        got = queues[c].drain_frames()
        assert got == want[c], c


def test_full_queue_holds_frames_until_room(B, S):
    """A batch whose frames do not fit a connection's queue keeps them and delivers them on a
    later poll (the reference would panic, repair_queue.go:53)."""
    k, m = 2, 1
    enc, _ = B.BatchEncoder.new(S.REED_SOLOMON_FEC_SCHEME, k, m, max_blocks=8)
    q = B.RepairQueue(max_len=2)
    mgr, _ = S.new_manager(S.REED_SOLOMON_FEC_SCHEME, k, m)
    for ssid in range(2 * 4):
        assert mgr.add_source_symbol_frame_batched(ssid, bytes([ssid]) * 50, enc, q) is None
    n, err = enc.drain()
    assert err == "repair queue full" and len(q) == 2
    got = q.drain_frames()
    n, err = enc.drain()
    assert err is None and len(q) == 2
    got += q.drain_frames()
    assert [f[0] for f in got] == [0, 1, 2, 3]
