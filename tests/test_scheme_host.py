"""Host-mirror logic without a GPU: block bookkeeping (block.go), manager bookkeeping
(manager.go) and every scheme error path of the reference's table tests that returns before
any arithmetic (reed_solomon_test.go, xor_test.go cases with wantErr or nil results)."""
import pytest

from scheme_util import block_from_case, needs_device, scheme_mod


@pytest.fixture(scope="module")
def S(fec):
    return scheme_mod()


def _scheme(S, case, kind):
    if kind == "xor":
        return S.xor_scheme()
    k, m = case["rs_new"] or (case["block"]["totNumSourceSymbols"], case["block"]["totNumRepairSymbols"])
    s, err = S.new_reed_solomon_scheme(k, m)
    assert err is None
    return s


@pytest.mark.parametrize("key,kind,method", [
    ("rs_repair", "rs", "repair_symbols"), ("rs_recover", "rs", "recover_symbol_payloads"),
    ("xor_repair", "xor", "repair_symbols"), ("xor_recover", "xor", "recover_symbol_payloads")])
def test_reference_cases_without_arithmetic(S, golden, key, kind, method):
    ran = 0
    for case in golden[key]:
        if needs_device(case):
            continue
        b = block_from_case(case["block"])
        got, err = getattr(_scheme(S, case, kind), method)(b)
        assert (err is not None) == case["wantErr"], (case["ref"], err)
        assert got is None, case["ref"]
        ran += 1
    assert ran >= 2


def test_error_texts_match_reference(S):
    b = S.Block.literal(tot_src=2, tot_rep=1, sources={1: (b"\x00\x01\x02", 3)})
    _, err = S.xor_scheme().repair_symbols(b)
    assert err == "block does not have enough source symbols to generate repair symbols"      # xor.go:16
    b = S.Block.literal(tot_src=2, tot_rep=2, sources={1: (b"abc", 3), 2: (b"def", 3)})
    _, err = S.xor_scheme().repair_symbols(b)
    assert err == "xor only supports 1 repair symbol. Expected 1, received 2"                   # xor.go:20
    b = S.Block.literal(tot_src=2, tot_rep=1, biggest=1435,
                        sources={1: (bytes(1435), 1435), 2: (bytes(1434), 1434)})
    rs, _ = S.new_reed_solomon_scheme(2, 1)
    _, err = rs.repair_symbols(b)
    assert err == "source symbol payload len is greater is too big for FEC headers. Max 1434 and got 1435"
    b = S.Block.literal(tot_src=2, tot_rep=1, sources={1: (b"\x00\x01\x02", 3)})
    _, err = rs.recover_symbol_payloads(b)
    assert err == "not enough present symbols to repair the missing ones"                      # :94
    # shard len beyond the payload's capacity (reed_solomon.go:81-84)
    b = S.Block.literal(tot_src=2, tot_rep=1, biggest=4, smallest=0, largest=1,
                        sources={0: (b"abcd", 4), 1: (b"ab", 1452)})
    _, err = rs.repair_symbols(b)
    assert err == "shard len (6) is greater than capacity of payload (4)"


def test_reed_solomon_new_validation(S):
    _, err = S.new_reed_solomon_scheme(0, 1)
    assert err and "less than one data shard" in err
    _, err = S.new_reed_solomon_scheme(200, 57)
    assert err and "256" in err
    s, err = S.new_reed_solomon_scheme(20, 10)
    assert err is None and s is not None


def test_block_bookkeeping(S):
    b = S.Block.new(2, 3, 2)                 # SSIDs [6, 8]
    err = b.add_source_symbol(9, b"x")
    assert err == "source symbol was provided to the wrong block. Expecting SID within the range [6, 8] and got 9"
    assert b.add_source_symbol(6, b"hello") is None
    assert b.add_source_symbol(6, b"hello world") is None       # duplicate ignored (block.go:63)
    assert b.biggest == 5 and b.get_source(6) == b"hello"
    assert b.add_source_symbol(7, b"a longer payload") is None
    assert b.biggest == 16
    assert not b.is_recoverable() and not b.is_complete()
    err = b.add_repair_symbol(3, 0, b"zz")
    assert err == "the repair symbol was provided to the wrong block. Expecting 2 and got 3"
    assert b.add_repair_symbol(2, 0, bytes(12)) is None
    assert b.biggest == 10                   # overwritten by len(repair) - 2 (block.go:82)
    assert b.is_recoverable() and not b.is_complete()
    assert b.add_source_symbol(8, b"z") is None
    assert b.is_complete()


def test_manager_factories_and_ssids(S):
    m, err = S.new_sender(S.FEC_DISABLED)
    assert m is None and err is None
    m, err = S.new_receiver(7)
    assert m is None and err == "unknown FEC scheme: 7"
    m, err = S.new_manager(S.XOR_FEC_SCHEME, -1, 1)
    assert m is None and err == "numTotSourceSymbols (-1) and numTotRepairSymbols (1) may not be negative"
    m, err = S.new_sender(S.REED_SOLOMON_FEC_SCHEME)
    assert err is None
    assert [m.next_ssid() for _ in range(4)] == [0, 1, 2, 3]
    assert m.block_id(19) == 0 and m.block_id(20) == 1 and m.block_id(45) == 2   # sid / 20


def test_receiver_source_path_and_processed_blocks(S):
    """HandleSourceSymbolFrame returns the payload, marks a complete block processed, and
    later symbols of a processed block are ignored (manager.go:200-227) — no arithmetic."""
    m, _ = S.new_receiver(S.XOR_FEC_SCHEME)
    got, err = m.handle_source_symbol_frame(0, b"first")
    assert (got, err) == (b"first", None)
    got, err = m.handle_source_symbol_frame(1, b"second")
    assert (got, err) == (b"second", None)            # block 0 now complete -> processed
    got, err = m.handle_repair_frame(0, 0, b"whatever")
    assert (got, err) == (None, None)                  # processed block: ignored
    got, err = m.handle_source_symbol_frame(0, b"again")
    assert (got, err) == (None, None)
    got, err = m.handle_repair_frame(5, 0, b"\x01\x02\x03")   # block 5: 1 repair < k=2
    assert (got, err) == (None, None)


def test_recover_on_source_flag_without_recovery(S):
    """The recover-on-source extension (off by default) changes nothing while no block becomes
    recoverable by a source: payloads come back, complete blocks are processed — no arithmetic."""
    m, _ = S.new_receiver(S.XOR_FEC_SCHEME)
    m.set_recover_on_source(True)
    assert m.handle_source_symbol_frame_recover(0, b"first") == (b"first", None, None)
    assert m.handle_source_symbol_frame_recover(1, b"second") == (b"second", None, None)
    assert m.handle_source_symbol_frame_recover(0, b"again") == (None, None, None)   # processed
    got, err = m.handle_repair_frame(5, 0, b"\x01\x02\x03")                          # 1 repair < k=2
    assert (got, err) == (None, None)
    m.set_recover_on_source(False)
    assert m.handle_source_symbol_frame_recover(12, b"x") == (b"x", None, None)
