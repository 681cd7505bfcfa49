"""Recover-on-source extension, default off.

The reference recovers a block only when a REPAIR frame makes it recoverable
(manager.go:181); a block whose repairs arrived before its last surviving source stays
unrecovered, because HandleSourceSymbolFrame only checks isComplete (manager.go:221-226).
With Manager.set_recover_on_source(True), the source arrival that makes the block
recoverable recovers it too. These tests drive shuffled arrivals (repairs before sources,
losses) through the per-block and the batched receivers and check the recovered payloads
against the senders' payloads, with the trigger rule modelled here in plain Python: flag off
must reproduce the reference's behaviour exactly, flag on must recover every recoverable,
incomplete block exactly once."""
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


def _arrivals(S, rng, sid, k, m, nblocks, loss):
    """Sender frames for nblocks blocks; per block a shuffled subset of its k + m symbols."""
    snd, _ = S.new_manager(sid, k, m)
    payloads, events = [], []
    for blk in range(nblocks):
        reps = []
        for j in range(k):
            p = rng.integers(0, 256, int(rng.choice([1, 90, 1200, 1434])), dtype=np.uint8).tobytes()
            payloads.append(p)
            fr, err = snd.add_source_symbol_frame(blk * k + j, p)
            assert err is None
            reps += fr or []
        ev = [("src", blk * k + j, payloads[blk * k + j]) for j in range(k)]
        ev += [("rep",) + tuple(r) for r in reps]
        ev = [e for e in ev if rng.random() >= loss]
        order = rng.permutation(len(ev))
        events += [ev[i] for i in order]
    return payloads, events


def _model(events, payloads, k, on_source):
    """The trigger rule: (block, recovered bytes) in the order recoveries fire."""
    src, rep, done, out = {}, {}, set(), []
    for e in events:
        blk = e[1] // k if e[0] == "src" else e[1]
        if blk in done:
            continue
        s, r = src.setdefault(blk, set()), rep.setdefault(blk, set())
        (s if e[0] == "src" else r).add(e[1] if e[0] == "src" else e[2])
        if len(s) == k:
            done.add(blk)
        elif len(s) + len(r) >= k and (e[0] == "rep" or on_source):
            missing = [blk * k + j for j in range(k) if blk * k + j not in s]
            out.append((blk, b"".join(payloads[i] for i in missing)))
            done.add(blk)
    return out


CASES = [("rs", 20, 10, 6, 0.2), ("rs", 8, 4, 24, 0.15), ("rs", 2, 1, 40, 0.2), ("xor", 2, 1, 40, 0.25)]


def _oracle_receiver(oracle, scheme, k, m, events, on):
    """The same arrivals through the oracle's manager (manager.go restated, CPU)."""
    rcv = oracle.Manager(scheme, k, m, recover_on_source=on)
    got = []
    for e in events:
        if e[0] == "src":
            _, rec, err = rcv.handle_source_symbol_frame(e[1], e[2])
            blk = e[1] // k
        else:
            rec, err = rcv.handle_repair_frame(e[1], e[2], e[3])
            blk = e[1]
        assert err is None
        if rec is not None:
            got.append((blk, rec))
    return got


@pytest.mark.parametrize("scheme,k,m,nblocks,loss", CASES)
@pytest.mark.parametrize("on", [False, True])
def test_per_block_receiver(S, oracle, scheme, k, m, nblocks, loss, on):
    rng = np.random.default_rng(1000 * k + m)
    sid = S.XOR_FEC_SCHEME if scheme == "xor" else S.REED_SOLOMON_FEC_SCHEME
    payloads, events = _arrivals(S, rng, sid, k, m, nblocks, loss)
    want = _model(events, payloads, k, on)
    assert _oracle_receiver(oracle, scheme, k, m, events, on) == want
    if on:
        assert len(want) > len(_model(events, payloads, k, False))   # the extension matters here
    rcv, _ = S.new_manager(sid, k, m)
    if on:
        rcv.set_recover_on_source(True)
    got = []
    for e in events:
        if e[0] == "src":
            p, rec, err = rcv.handle_source_symbol_frame_recover(e[1], e[2])
            assert err is None and p in (e[2], None)
            if rec is not None:
                got.append((e[1] // k, rec))
        else:
            rec, err = rcv.handle_repair_frame(e[1], e[2], e[3])
            assert err is None
            if rec is not None:
                got.append((e[1], rec))
    assert got == want


@pytest.mark.parametrize("scheme,k,m,nblocks,loss", CASES)
def test_batched_receiver(B, S, oracle, scheme, k, m, nblocks, loss):
    """Same arrivals through HandleSourceSymbolFrameBatched / HandleRepairFrameBatched with the
    flag on: the RecoveredQueue holds exactly the per-block path's recoveries, in order."""
    rng = np.random.default_rng(1000 * k + m)
    sid = S.XOR_FEC_SCHEME if scheme == "xor" else S.REED_SOLOMON_FEC_SCHEME
    payloads, events = _arrivals(S, rng, sid, k, m, nblocks, loss)
    want = _model(events, payloads, k, True)
    assert _oracle_receiver(oracle, scheme, k, m, events, True) == want
    dec, err = B.BatchDecoder.new(sid, k, m, max_blocks=5)
    assert err is None
    rcv, _ = S.new_manager(sid, k, m)
    rcv.set_recover_on_source(True)
    q = B.RecoveredQueue()
    for i, e in enumerate(events):
        if e[0] == "src":
            p, err = rcv.handle_source_symbol_frame_batched(e[1], e[2], dec, q)
            assert err is None and p in (e[2], None)
        else:
            assert rcv.handle_repair_frame_batched(e[1], e[2], e[3], dec, q) is None
        if i % 13 == 7:
            assert dec.poll()[1] is None
    assert dec.drain()[1] is None
    assert q.drain() == want
