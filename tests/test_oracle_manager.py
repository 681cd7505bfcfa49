"""The oracle's manager (oracle.Manager, manager.go restated) on the CPU: a sender's frames
through a lossy channel into a receiver recover exactly the lost payloads, for the
reference's factory codes and the bench shapes; and the manager's bookkeeping rules
(processed blocks ignored, out-of-range SSIDs rejected). The reference has no manager tests
(SURVEY.md §4); the scheme functions underneath are pinned by test_oracle_golden.py."""
import numpy as np
import pytest


@pytest.mark.parametrize("scheme,k,m", [("rs", 20, 10), ("rs", 8, 4), ("rs", 2, 1), ("xor", 2, 1), ("xor", 5, 1)])
def test_sender_to_lossy_receiver(oracle, scheme, k, m):
    rng = np.random.default_rng(k * 31 + m)
    snd, rcv = oracle.Manager(scheme, k, m), oracle.Manager(scheme, k, m)
    nblocks = 6
    pl = [rng.integers(0, 256, int(rng.integers(1, 1435)), dtype=np.uint8).tobytes() for _ in range(nblocks * k)]
    frames = []
    for ssid, p in enumerate(pl):
        fr, err = snd.add_source_symbol_frame(ssid, p)
        assert err is None
        frames.append(fr)
    for blk in range(nblocks):
        assert frames[blk * k + k - 1] is not None and all(f is None for f in frames[blk * k:blk * k + k - 1])
        assert [f[1] for f in frames[blk * k + k - 1]] == list(range(m))
    got = {}
    for blk in range(nblocks):
        lost = set(rng.choice(k, size=min(m, 1 + blk % m), replace=False).tolist())
        for j in range(k):
            if j not in lost:
                p, rec, err = rcv.handle_source_symbol_frame(blk * k + j, pl[blk * k + j])
                assert err is None and p == pl[blk * k + j] and rec is None
        for (bid, pid, payload) in frames[blk * k + k - 1]:
            rec, err = rcv.handle_repair_frame(bid, pid, payload)
            assert err is None
            if rec is not None:
                got[bid] = rec
        assert got[blk] == b"".join(pl[blk * k + j] for j in sorted(lost))


def test_manager_bookkeeping(oracle):
    mg = oracle.Manager("rs", 2, 1)
    assert mg.add_source_symbol_frame(0, b"ab") == (None, None)
    fr, err = mg.add_source_symbol_frame(1, b"c")
    assert err is None and len(fr) == 1
    assert mg.add_source_symbol_frame(1, b"zz") == (None, None)        # processed: ignored
    rcv = oracle.Manager("rs", 2, 1)
    rec, err = rcv.handle_repair_frame(0, 0, fr[0][2])
    assert (rec, err) == (None, None)                                  # not yet recoverable
    p, rec, err = rcv.handle_source_symbol_frame(1, b"c")
    assert p == b"c" and rec is None and err is None                   # reference: no recovery on source
    rcv2 = oracle.Manager("rs", 2, 1, recover_on_source=True)
    rcv2.handle_repair_frame(0, 0, fr[0][2])
    p, rec, err = rcv2.handle_source_symbol_frame(1, b"c")
    assert rec == b"ab" and err is None                                # the optional extension
