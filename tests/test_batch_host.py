"""Sender-side batching layer without a GPU: repair_queue.go semantics (Add / Peek / Pop, the
32-frame limit, hasData, CloseWithError) and the BatchEncoder checks that must return the
reference's repairSymbols errors before any device work."""
import importlib

import pytest


@pytest.fixture(scope="module")
def B(fec):
    return importlib.import_module("0xfec_amd.batch")


@pytest.fixture(scope="module")
def S(fec):
    return importlib.import_module("0xfec_amd.scheme")


def test_repair_queue_fifo_limit_and_has_data(B):
    q = B.RepairQueue()
    assert q.peek() is None and len(q) == 0
    for i in range(32):                       # maxRepairSendQueueLen (repair_queue.go:14)
        assert q.add(7, i, bytes([i]) * 3) is None
    assert q.has_data_calls == 32             # hasData() after every Add (repair_queue.go:48)
    assert q.add(7, 32, b"x") == "repair queue full"   # the reference panics here
    assert len(q) == 32
    for i in range(32):
        assert q.peek() == (7, i, bytes([i]) * 3)
        assert q.peek() == (7, i, bytes([i]) * 3)   # Peek does not consume
        q.pop()
    assert q.peek() is None
    q.pop()                                    # Pop on empty: no-op (ringbuffer PopFront guard)
    assert q.add(1, 0, b"") is None and q.peek() == (1, 0, b"")


def test_repair_queue_custom_limit_and_close(B):
    q = B.RepairQueue(max_len=3)
    for i in range(3):
        assert q.add(0, i, b"a") is None
    assert q.add(0, 3, b"a") == "repair queue full"
    q.close_with_error("connection closed")
    q.pop()
    assert q.add(0, 9, b"a") == "connection closed"


def test_batch_encoder_construction_errors(B, S):
    enc, err = B.BatchEncoder.new(S.XOR_FEC_SCHEME, 2, 2)
    assert enc is None and "xor only supports 1 repair symbol" in err
    enc, err = B.BatchEncoder.new(S.REED_SOLOMON_FEC_SCHEME, 0, 2)
    assert enc is None and err
    enc, err = B.BatchEncoder.new(S.REED_SOLOMON_FEC_SCHEME, 8, 4, max_blocks=0)
    assert enc is None and err
    enc, err = B.BatchEncoder.new(S.FEC_DISABLED, 2, 1)
    assert enc is None and err


def test_batch_encoder_validates_before_device_work(B, S):
    """Submit returns repairSymbols' own errors (reed_solomon.go:27-33, xor.go:15-25) with no
    device: the checks run before staging memory is allocated."""
    enc, err = B.BatchEncoder.new(S.REED_SOLOMON_FEC_SCHEME, 2, 1)
    assert err is None
    q = B.RepairQueue()
    b = S.Block.literal(tot_src=2, tot_rep=1, sources={0: (b"\x01\x02", 1452)})
    assert enc.submit(b, q) == "block does not have enough source symbols to generate repair symbols"
    b = S.Block.literal(tot_src=2, tot_rep=1, biggest=1435, smallest=0, largest=1,
                        sources={0: (b"\x01" * 10, 1452), 1: (b"\x02" * 10, 1452)})
    assert "1435" in enc.submit(b, q)
    xenc, err = B.BatchEncoder.new(S.XOR_FEC_SCHEME, 2, 1)
    assert err is None
    b = S.Block.literal(tot_src=2, tot_rep=1, sources={5: (b"\x01", 1452)})
    assert xenc.submit(b, q) == "block does not have enough source symbols to generate repair symbols"
    assert len(q) == 0 and enc.staged == 0 and enc.in_flight == 0


def test_batch_decoder_validates_before_device_work(B, S):
    dec, err = B.BatchDecoder.new(S.REED_SOLOMON_FEC_SCHEME, 2, 1)
    assert err is None
    q = B.RecoveredQueue()
    b = S.Block.literal(tot_src=2, tot_rep=1, sources={0: (b"\x01\x02", 1452)})
    staged, err = dec.submit(b, q)
    assert not staged and err == "not enough present symbols to repair the missing ones"
    # complete block: the reference's nil, nil — nothing staged, no error, no device needed
    b = S.Block.literal(tot_src=2, tot_rep=1, smallest=0, largest=1,
                        sources={0: (b"\x01", 1452), 1: (b"\x02", 1452)})
    staged, err = dec.submit(b, q)
    assert not staged and err is None and len(q) == 0
    d2, err = B.BatchDecoder.new(S.XOR_FEC_SCHEME, 2, 3)
    assert d2 is None and "xor only supports 1 repair symbol" in err
