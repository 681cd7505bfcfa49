"""Pin the CPU oracle to the reference's own golden vectors (no GPU).

Every case of internal/fec/reed_solomon_test.go and internal/fec/xor_test.go is replayed
through the oracle's restatement of the scheme layer (oracle/oracle.py) and must give the
reference's expected bytes / error outcome. Fixtures: tests/golden/reference_cases.json
(text-extracted by tests/golden/extract_golden.py).
"""
import numpy as np
import pytest


def _cases(golden, key):
    return [pytest.param(c, id=c["ref"]) for c in golden[key]]


def _frames(want):
    return [(f["BlockID"], f["ParityID"], bytes.fromhex(f["Payload"]["hex"])) for f in want["frames"]]


def test_fixture_inventory(golden):
    assert len(golden["rs_repair"]) == 4
    assert len(golden["rs_recover"]) == 4
    assert len(golden["xor_repair"]) == 6
    assert len(golden["xor_recover"]) == 4


def test_rs_repair_golden(oracle, golden):
    for c in golden["rs_repair"]:
        b = oracle.block_from_fixture(c["block"])
        k, m = c["rs_new"] or (b.tot_src, b.tot_rep)
        got, err = oracle.rs_repair_symbols(b, k, m)
        assert (err is not None) == c["wantErr"], c["ref"]
        if not c["wantErr"]:
            assert got == _frames(c["want"]), c["ref"]


def test_rs_recover_golden(oracle, golden):
    for c in golden["rs_recover"]:
        b = oracle.block_from_fixture(c["block"])
        k, m = c["rs_new"] or (b.tot_src, b.tot_rep)
        got, err = oracle.rs_recover_symbol_payloads(b, k, m)
        assert (err is not None) == c["wantErr"], c["ref"]
        want = None if c["want"] is None else bytes.fromhex(c["want"]["bytes"])
        assert got == want, c["ref"]


def test_xor_repair_golden(oracle, golden):
    for c in golden["xor_repair"]:
        b = oracle.block_from_fixture(c["block"])
        got, err = oracle.xor_repair_symbols(b)
        assert (err is not None) == c["wantErr"], c["ref"]
        if not c["wantErr"]:
            assert got == _frames(c["want"]), c["ref"]


def test_xor_recover_golden(oracle, golden):
    for c in golden["xor_recover"]:
        b = oracle.block_from_fixture(c["block"])
        got, err = oracle.xor_recover_symbol_payloads(b)
        assert (err is not None) == c["wantErr"], c["ref"]
        want = None if c["want"] is None else bytes.fromhex(c["want"]["bytes"])
        assert got == want, c["ref"]


def test_systematic_rows_known_answers(oracle):
    """SURVEY.md §8a parity rows of the klauspost default matrix (pinned transitively by the
    6/2 and 20/10 goldens above)."""
    assert oracle.build_matrix(2, 3)[2].tolist() == [0x03, 0x02]
    m = oracle.build_matrix(6, 8)
    assert m[6].tolist() == [7, 6, 5, 4, 3, 2]
    assert m[7].tolist() == [6, 7, 4, 5, 2, 3]
    m = oracle.build_matrix(8, 12)
    assert bytes(m[8]).hex() == "1a84ba33e710c627"
    assert bytes(m[9]).hex() == "841a33ba10e727c6"
    assert bytes(m[10]).hex() == "ba331a84c627e710"
    assert bytes(m[11]).hex() == "33ba841a27c610e7"
    assert bytes(oracle.build_matrix(16, 24)[16]).hex() == "21b5f685df02b7873edd4aa48dda6130"
    for k, n in [(2, 3), (8, 12), (16, 24), (20, 30)]:
        mat = oracle.build_matrix(k, n)
        assert (mat[:k] == np.eye(k, dtype=np.uint8)).all()


def test_gf_field(oracle):
    assert oracle.gf_mul(2, 0x80) == 0x1D
    assert oracle.gf_mul(0, 7) == 0 and oracle.gf_mul(1, 0xAB) == 0xAB
    for a in range(1, 256):
        inv = int(oracle.lib().fo_gf_div(1, a))
        assert oracle.gf_mul(a, inv) == 1


def test_batch_roundtrip_mds(oracle):
    """Any k of the n shards rebuild the data (MDS), for every erasure pattern of RS(4,6)."""
    import itertools
    rng = np.random.default_rng(0x0FEC)
    k, m, S = 4, 2, 40
    n = k + m
    pats = [p for r in range(0, m + 1) for p in itertools.combinations(range(n), r)]
    B = len(pats)
    shards = np.zeros((B, n, S), dtype=np.uint8)
    shards[:, :k] = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    oracle.rs_encode(k, m, shards)
    ref = shards.copy()
    masks = np.array([((1 << n) - 1) & ~sum(1 << i for i in p) for p in pats], dtype=np.uint32)
    for b, p in enumerate(pats):
        for i in p:
            shards[b, i] = 0
    st = oracle.rs_reconstruct(k, m, shards, masks)
    assert (st == 0).all()
    assert (shards[:, :k] == ref[:, :k]).all()
    bad = np.array([(1 << (k - 1)) - 1], dtype=np.uint32)
    assert oracle.rs_reconstruct(k, m, shards[:1].copy(), bad)[0] == -1
