"""GPU parity of the batching layer against the CPU oracle (oracle.Manager: manager.go restated
over the oracle's repairSymbols / recoverSymbolPayloads): the repair frames a connection's
RepairQueue receives from the batched sender, and the payloads its RecoveredQueue receives from
the batched receiver, equal in order and byte for byte what the oracle's manager returns for
the same symbols — and what the per-block HIP path returns — across batch boundaries,
double-buffered batches, mixed symbol lengths and several connections sharing one encoder."""
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


@pytest.mark.parametrize("zc", [0, 1 << 30])   # knob bat_zc: the copy form, every set zero-copy
@pytest.mark.parametrize("scheme,k,m,max_blocks,lens", [
    ("rs", 20, 10, 4, [1200]),                       # the reference's RS factory code
    ("rs", 8, 4, 5, [1, 17, 600, 1200, 1434]),       # mixed lengths: slot-overflow flushes
    ("rs", 2, 1, 64, [1200, 1434]),
    ("xor", 2, 1, 3, [1, 100, 1200, 1434]),          # the reference's XOR factory code
])
def test_batched_frames_equal_per_block_frames(B, S, oracle, tune, scheme, k, m, max_blocks, lens, zc):
    tune(bat_zc=zc)
    rng = np.random.default_rng(k * 100 + max_blocks)
    sid = S.XOR_FEC_SCHEME if scheme == "xor" else S.REED_SOLOMON_FEC_SCHEME
    nconn, nblocks = 3, 7
    streams = _streams(rng, nconn, nblocks, k, lens)
    # the oracle's manager (CPU)
    orc = []
    for pl in streams:
        mgr = oracle.Manager(scheme, k, m)
        frames = []
        for ssid, p in enumerate(pl):
            fr, err = mgr.add_source_symbol_frame(ssid, p)
            assert err is None
            frames += fr or []
        orc.append(frames)
    # per-block HIP path
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
    assert want == orc
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
    assert err == "repair queue full" and len(q) == 2 and enc.backlog == 2
    got = q.drain_frames()
    n, err = enc.drain()
    assert err is None and len(q) == 2 and enc.backlog == 0
    got += q.drain_frames()
    assert [f[0] for f in got] == [0, 1, 2, 3]


def test_submit_never_fails_on_a_full_queue(B, S, oracle):
    """Backpressure from an earlier batch must not fail Submit (the block would never be
    encoded: the manager drops complete blocks, manager.go:145-153): small batches flushed by
    Submit itself while the connection's queue is full; every block's frames arrive, in order,
    equal to the oracle's repairSymbols."""
    k, m = 8, 4
    enc, _ = B.BatchEncoder.new(S.REED_SOLOMON_FEC_SCHEME, k, m, max_blocks=2)
    q = B.RepairQueue(max_len=m)          # room for one block's frames
    mgr, _ = S.new_manager(S.REED_SOLOMON_FEC_SCHEME, k, m)
    rng = np.random.default_rng(77)
    nblocks = 9
    pl = [rng.integers(0, 256, int(rng.integers(1, 1435)), dtype=np.uint8).tobytes() for _ in range(nblocks * k)]
    got = []
    for ssid, p in enumerate(pl):
        # every Submit (on each block's k-th symbol) may flush and retire a batch into a full queue
        assert mgr.add_source_symbol_frame_batched(ssid, p, enc, q) is None
        if ssid % (3 * k) == 3 * k - 1:
            got += q.drain_frames()
    while True:
        n, err = enc.drain()
        got += q.drain_frames()
        if err is None:
            break
        assert err == "repair queue full"
    orc = oracle.Manager("rs", k, m)
    want = sum((orc.add_source_symbol_frame(ssid, p)[0] or [] for ssid, p in enumerate(pl)), [])
    assert len(want) == nblocks * m and got == want


# zc: the decoder's sets are coded straight from / into their pinned buffers (knob bat_zc) when
# their input is at most this many bytes (1 << 30: every set; 0: the copy form)
@pytest.mark.parametrize("zc", [0, 1 << 30])
@pytest.mark.parametrize("scheme,k,m,max_blocks,lens,loss", [
    ("rs", 20, 10, 4, [1200], 0.15),
    ("rs", 8, 4, 3, [1, 17, 600, 1200, 1434], 0.25),
    ("rs", 2, 1, 64, [1200, 1434], 0.3),
    ("xor", 2, 1, 3, [1, 100, 1200, 1434], 0.3),
])
def test_batched_recovery_equals_per_block_recovery(B, S, oracle, tune, scheme, k, m, max_blocks, lens, loss, zc):
    """Receiver: the payloads HandleRepairFrame returns per block (manager.go:160-198) equal,
    in order, those the batched path delivers to the connection's RecoveredQueue, under random
    source and repair losses (some blocks unrecoverable, some complete before any repair)."""
    tune(bat_zc=zc)
    rng = np.random.default_rng(k * 7 + max_blocks)
    sid = S.XOR_FEC_SCHEME if scheme == "xor" else S.REED_SOLOMON_FEC_SCHEME
    nconn, nblocks = 3, 9
    streams = _streams(rng, nconn, nblocks, k, lens)
    # the senders' frames, then a loss pattern per connection
    arrivals = []
    for pl in streams:
        snd, _ = S.new_manager(sid, k, m)
        ev = []
        for blk in range(nblocks):
            reps = []
            for j in range(k):
                ssid = blk * k + j
                fr, err = snd.add_source_symbol_frame(ssid, pl[ssid])
                assert err is None
                if rng.random() >= loss:
                    ev.append(("src", ssid, pl[ssid]))
                reps += fr or []
            for (bid, pid, payload) in reps:
                if rng.random() >= loss / 2:
                    ev.append(("rep", bid, pid, payload))
        arrivals.append(ev)
    # per-block receivers
    want = []
    for ev in arrivals:
        rcv, _ = S.new_manager(sid, k, m)
        got = []
        for e in ev:
            if e[0] == "src":
                _, err = rcv.handle_source_symbol_frame(e[1], e[2])
            else:
                rec, err = rcv.handle_repair_frame(e[1], e[2], e[3])
                if rec is not None:
                    got.append((e[1], rec))
            assert err is None
        want.append(got)
    assert sum(len(w) for w in want) > 0
    # the oracle's receivers (CPU)
    for c, ev in enumerate(arrivals):
        rcv = oracle.Manager(scheme, k, m)
        got = []
        for e in ev:
            if e[0] == "src":
                _, _, err = rcv.handle_source_symbol_frame(e[1], e[2])
            else:
                rec, err = rcv.handle_repair_frame(e[1], e[2], e[3])
                if rec is not None:
                    got.append((e[1], rec))
            assert err is None
        assert got == want[c], c
    # batched receivers sharing one decoder, arrivals interleaved across connections
    dec, err = B.BatchDecoder.new(sid, k, m, max_blocks=max_blocks)
    assert err is None
    rcvs = [S.new_manager(sid, k, m)[0] for _ in range(nconn)]
    queues = [B.RecoveredQueue() for _ in range(nconn)]
    for i in range(max(len(ev) for ev in arrivals)):
        for c in range(nconn):
            if i >= len(arrivals[c]):
                continue
            e = arrivals[c][i]
            if e[0] == "src":
                _, err = rcvs[c].handle_source_symbol_frame(e[1], e[2])
            else:
                err = rcvs[c].handle_repair_frame_batched(e[1], e[2], e[3], dec, queues[c])
            assert err is None
        if i % 11 == 5:
            assert dec.poll()[1] is None
    n, err = dec.drain()
    assert err is None and dec.staged == 0 and dec.in_flight == 0
    for c in range(nconn):
        assert queues[c].drain() == want[c], c


@pytest.mark.parametrize("scheme,k,m", [("rs", 20, 10), ("rs", 8, 4), ("xor", 2, 1)])
def test_submit_payloads_equals_manager_path(B, S, oracle, scheme, k, m):
    """Zero-copy staging of source payloads (fec_wire.h) yields the frames the per-block
    manager path returns for the same symbols."""
    W = importlib.import_module("0xfec_amd.wire")
    rng = np.random.default_rng(5 * k)
    sid = S.XOR_FEC_SCHEME if scheme == "xor" else S.REED_SOLOMON_FEC_SCHEME
    nblocks = 11
    pl = _streams(rng, 1, nblocks, k, [1, 33, 700, 1200, 1434])[0]
    mgr, _ = S.new_manager(sid, k, m)
    want = []
    for ssid, p in enumerate(pl):
        fr, err = mgr.add_source_symbol_frame(ssid, p)
        assert err is None
        want += fr or []
    orc = oracle.Manager(scheme, k, m)
    assert want == sum((orc.add_source_symbol_frame(ssid, p)[0] or [] for ssid, p in enumerate(pl)), [])
    enc, _ = B.BatchEncoder.new(sid, k, m, max_blocks=4)
    q = B.RepairQueue(max_len=nblocks * m)
    for blk in range(nblocks):
        assert W.submit_payloads(enc, blk, pl[blk * k:(blk + 1) * k], q) is None
    assert enc.drain()[1] is None
    assert q.drain_frames() == want


@pytest.mark.parametrize("rlen", [1441, 1446, 1452])
def test_long_repair_payload_batched_equals_per_block(B, S, oracle, rlen):
    """XOR recovery accepts repair payloads up to a packet buffer (1452 B, xor.go:76-86): the
    batched receiver must stage them like the per-block path and the oracle."""
    k, m = 2, 1
    rng = np.random.default_rng(rlen)
    big = rlen - 2                       # the receiver's biggest = len(repair) - 2 (block.go:82)
    src = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
    lost = rng.integers(0, 256, big, dtype=np.uint8).tobytes()
    rep = bytearray(rlen)                # xor framing of both payloads at `big` (xor.go:44-56)
    for p in (src, lost):
        for i, v in enumerate(p):
            rep[i] ^= v
        rep[big] ^= len(p) >> 8
        rep[big + 1] ^= len(p) & 0xFF
    rep = bytes(rep)
    orc = oracle.Manager("xor", k, m)
    orc.handle_source_symbol_frame(0, src)
    want, err = orc.handle_repair_frame(0, 0, rep)
    assert err is None and want == lost
    rcv, _ = S.new_manager(S.XOR_FEC_SCHEME, k, m)
    rcv.handle_source_symbol_frame(0, src)
    got, err = rcv.handle_repair_frame(0, 0, rep)
    assert err is None and got == want
    dec, _ = B.BatchDecoder.new(S.XOR_FEC_SCHEME, k, m, max_blocks=4)
    rcv2, _ = S.new_manager(S.XOR_FEC_SCHEME, k, m)
    q = B.RecoveredQueue()
    rcv2.handle_source_symbol_frame(0, src)
    assert rcv2.handle_repair_frame_batched(0, 0, rep, dec, q) is None
    assert dec.drain()[1] is None
    assert q.drain() == [(0, want)]
