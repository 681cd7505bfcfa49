"""The reference's own table tests, replayed through the host mirror of internal/fec and the
GPU codec (reed_solomon_test.go, xor_test.go), plus manager-level sender -> lossy channel ->
receiver runs checked against the CPU oracle's restatement of the same Go code."""
import numpy as np
import pytest

from scheme_util import block_from_case, want_frames, scheme_mod

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def S(fec):
    import torch
    assert torch.cuda.is_available()
    return scheme_mod()


def _rs(S, case):
    k, m = case["rs_new"] or (case["block"]["totNumSourceSymbols"], case["block"]["totNumRepairSymbols"])
    s, err = S.new_reed_solomon_scheme(k, m)
    assert err is None
    return s


def test_reed_solomon_repair_symbols_golden(S, golden):          # reed_solomon_test.go:12-222
    for case in golden["rs_repair"]:
        got, err = _rs(S, case).repair_symbols(block_from_case(case["block"]))
        assert (err is not None) == case["wantErr"], case["ref"]
        if not case["wantErr"]:
            assert got == want_frames(case["want"]), case["ref"]


def test_reed_solomon_recover_symbol_payloads_golden(S, golden):  # reed_solomon_test.go:234-371
    for case in golden["rs_recover"]:
        got, err = _rs(S, case).recover_symbol_payloads(block_from_case(case["block"]))
        assert (err is not None) == case["wantErr"], case["ref"]
        want = None if case["want"] is None else bytes.fromhex(case["want"]["bytes"])
        assert got == want, case["ref"]


def test_xor_repair_symbols_golden(S, golden):                    # xor_test.go:11-164
    for case in golden["xor_repair"]:
        got, err = S.xor_scheme().repair_symbols(block_from_case(case["block"]))
        assert (err is not None) == case["wantErr"], case["ref"]
        if not case["wantErr"]:
            assert got == want_frames(case["want"]), case["ref"]


def test_xor_recover_symbol_payloads_golden(S, golden):           # xor_test.go:186-283
    for case in golden["xor_recover"]:
        b = block_from_case(case["block"])
        got, err = S.xor_scheme().recover_symbol_payloads(b)
        assert (err is not None) == case["wantErr"], case["ref"]
        want = None if case["want"] is None else bytes.fromhex(case["want"]["bytes"])
        assert got == want, case["ref"]
        if want is not None:
            assert b.is_complete()                                 # recovered symbol stored (xor.go:91-96)


@pytest.mark.parametrize("k,m", [(2, 1), (6, 2), (8, 4), (20, 10), (16, 8)])
def test_random_blocks_match_oracle_scheme(S, oracle, k, m):
    """Variable payload lengths (zero padding + length trailer), every loss count <= m."""
    rng = np.random.default_rng(1000 + k)
    s, _ = S.new_reed_solomon_scheme(k, m)
    for trial in range(6):
        lens = rng.integers(1, 1435, k)
        biggest = int(lens.max())
        payloads = {20 + i: bytes(rng.integers(0, 256, int(lens[i]), dtype=np.uint8)) for i in range(k)}
        ob = oracle.Block(id=1, tot_src=k, tot_rep=m, biggest=biggest, smallest=20, largest=20 + k - 1,
                          sources={sid: oracle.Payload(p, 1452) for sid, p in payloads.items()})
        want, werr = oracle.rs_repair_symbols(ob, k, m)
        gb = S.Block.literal(id=1, tot_src=k, tot_rep=m, biggest=biggest, smallest=20, largest=20 + k - 1,
                             sources={sid: (p, 1452) for sid, p in payloads.items()})
        got, err = s.repair_symbols(gb)
        assert werr is None and err is None and got == want
        lost = set(rng.choice(k, size=min(m, int(rng.integers(1, m + 1))), replace=False).tolist())
        keep_rep = sorted(rng.choice(m, size=len(lost), replace=False).tolist())
        rb_src = {sid: p for sid, p in payloads.items() if sid - 20 not in lost}
        ob2 = oracle.Block(id=1, tot_src=k, tot_rep=m, biggest=biggest, smallest=20, largest=20 + k - 1,
                           sources={sid: oracle.Payload(p, 1452) for sid, p in rb_src.items()},
                           repairs={pid: oracle.Payload(want[pid][2]) for pid in keep_rep})
        wrec, werr = oracle.rs_recover_symbol_payloads(ob2, k, m)
        gb2 = S.Block.literal(id=1, tot_src=k, tot_rep=m, biggest=biggest, smallest=20, largest=20 + k - 1,
                              sources={sid: (p, 1452) for sid, p in rb_src.items()},
                              repairs={pid: want[pid][2] for pid in keep_rep})
        grec, gerr = s.recover_symbol_payloads(gb2)
        assert werr is None and gerr is None
        assert grec == wrec == b"".join(payloads[20 + i] for i in sorted(lost))


def test_manager_xor_sender_receiver(S):
    """NewSender/NewReceiver(XOR): (2,1) blocks; lose one source per block, recover it."""
    snd, _ = S.new_sender(S.XOR_FEC_SCHEME)
    rcv, _ = S.new_receiver(S.XOR_FEC_SCHEME)
    rng = np.random.default_rng(5)
    for blk in range(6):
        p = [bytes(rng.integers(0, 256, int(rng.integers(1, 1435)), dtype=np.uint8)) for _ in range(2)]
        s0, s1 = snd.next_ssid(), snd.next_ssid()
        r0, err = snd.add_source_symbol_frame(s0, p[0])
        assert (r0, err) == (None, None)
        rep, err = snd.add_source_symbol_frame(s1, p[1])
        assert err is None and len(rep) == 1 and rep[0][:2] == (blk, 0)
        lost = blk % 2
        got, err = rcv.handle_source_symbol_frame([s0, s1][1 - lost], p[1 - lost])
        assert (got, err) == (p[1 - lost], None)
        rec, err = rcv.handle_repair_frame(rep[0][0], rep[0][1], rep[0][2])
        assert err is None and rec == p[lost]


def test_manager_reed_solomon_20_10(S, oracle):
    """NewSender/NewReceiver(ReedSolomon): RS(20,10) (manager.go:77-90). Up to 10 losses."""
    snd, _ = S.new_sender(S.REED_SOLOMON_FEC_SCHEME)
    rcv, _ = S.new_receiver(S.REED_SOLOMON_FEC_SCHEME)
    rng = np.random.default_rng(20)
    for blk in range(3):
        payloads = [bytes(rng.integers(0, 256, int(rng.integers(500, 1435)), dtype=np.uint8)) for _ in range(20)]
        ssids = [snd.next_ssid() for _ in range(20)]
        reps = None
        for sid, p in zip(ssids, payloads):
            r, err = snd.add_source_symbol_frame(sid, p)
            assert err is None
            if r:
                reps = r
        assert reps is not None and len(reps) == 10
        lost = sorted(rng.choice(20, size=3 + 3 * blk, replace=False).tolist())
        for i, (sid, p) in enumerate(zip(ssids, payloads)):
            if i not in lost:
                got, err = rcv.handle_source_symbol_frame(sid, p)
                assert err is None and got == p
        out = None
        for bid, pid, rp in reps[:len(lost)]:
            out, err = rcv.handle_repair_frame(bid, pid, rp)
            assert err is None
        assert out == b"".join(payloads[i] for i in lost)


def test_config1_plumbing_rs23_one_block(S, oracle):
    """BASELINE.json config #1: RS rate-2/3 (k=2, n=3), one block of two 1200-B symbols. The
    repair is row `03 02` of the default matrix applied to the framed shards;
    losing shard 0 and recovering it returns the 1200-B payload (reed_solomon.go:128-133)."""
    rng = np.random.default_rng(0x0FEC)
    p = [bytes(rng.integers(0, 256, 1200, dtype=np.uint8)) for _ in range(2)]
    s, err = S.new_reed_solomon_scheme(2, 1)
    assert err is None
    b = S.Block.literal(id=0, tot_src=2, tot_rep=1, biggest=1200, smallest=0, largest=1,
                        sources={0: (p[0], 1452), 1: (p[1], 1452)})
    frames, err = s.repair_symbols(b)
    assert err is None and len(frames) == 1 and frames[0][:2] == (0, 0)
    shards = [np.frombuffer(x + bytes([0x04, 0xB0]), dtype=np.uint8) for x in p]   # trailer 1200 = 0x04B0
    t3, t2 = (np.array([oracle.gf_mul(c, x) for x in range(256)], dtype=np.uint8) for c in (3, 2))
    want = bytes(t3[shards[0]] ^ t2[shards[1]])
    assert frames[0][2] == want and len(want) == 1202
    rb = S.Block.literal(id=0, tot_src=2, tot_rep=1, biggest=1200, smallest=0, largest=1,
                         sources={1: (p[1], 1452)}, repairs={0: frames[0][2]})
    got, err = s.recover_symbol_payloads(rb)
    assert err is None and got == p[0]
