"""The dyadic structure the fixed-shape encode relies on (fec_kernels.hip, "dyadic encode";
leaf tables from fec_capi.cpp dyadic_leaves()), checked on the CPU against the oracle's
restatement of klauspost's buildMatrix (oracle/fec_oracle.c):

  - for k and m powers of two (m <= k), parity row i, column j of the systematic matrix is
    g(i ^ j) with g = parity row 0;
  - the split-recursive product conv(C, D) = (P ^ Q, R ^ P ^ Q) over the leaf constants, in the
    order the host emits them (P's leaves, Q's, R's), gives the same parity bytes as the
    matrix product, for every byte value.
Parity of the GPU kernel itself is tests/test_gpu_codec.py (encode variants)."""
import numpy as np
import pytest

POW2_SHAPES = [(2, 1), (4, 2), (8, 4), (16, 8), (8, 2), (16, 4), (32, 16), (64, 32)]


def leaves(c):
    """dyadic_leaves() restated for one group's constants c (len 2^b) -> 3^b leaf constants."""
    if len(c) == 1:
        return [c[0]]
    h = len(c) // 2
    lo, hi = c[:h], c[h:]
    return leaves(lo) + leaves(hi) + leaves([a ^ b for a, b in zip(lo, hi)])


def conv(oracle, d, t):
    """Y[i] = sum_l C[l ^ i] * d[l] from the leaf constants t of C (the kernel's dy_conv)."""
    if len(d) == 1:
        return [oracle.gf_mul(t[0], d[0])]
    h, L = len(d) // 2, len(t) // 3
    P = conv(oracle, d[:h], t[:L])
    Q = conv(oracle, d[h:], t[L:2 * L])
    R = conv(oracle, [a ^ b for a, b in zip(d[:h], d[h:])], t[2 * L:])
    return [p ^ q for p, q in zip(P, Q)] + [r ^ p ^ q for r, p, q in zip(R, P, Q)]


@pytest.mark.parametrize("k,m", POW2_SHAPES)
def test_systematic_matrix_is_dyadic(oracle, k, m):
    M = oracle.build_matrix(k, k + m)
    g = M[k]
    for i in range(m):
        for j in range(k):
            assert M[k + i, j] == g[i ^ j], (k, m, i, j)


def test_rs_8_12_rows_match_survey_constants(oracle):
    """SURVEY.md §8a lists RS(8,12)'s parity rows; they are the XOR-shifts of row 0."""
    M = oracle.build_matrix(8, 12)
    assert bytes(M[8]).hex() == "1a84ba33e710c627"
    assert [bytes(M[8 + i]).hex() for i in range(4)] == [bytes(M[8][[j ^ i for j in range(8)]]).hex()
                                                       for i in range(4)]


@pytest.mark.parametrize("k,m", [(2, 1), (4, 2), (8, 4), (16, 8), (16, 4)])
def test_split_recursive_product_equals_matrix(oracle, k, m):
    M = oracle.build_matrix(k, k + m)
    g = [int(v) for v in M[k]]
    tabs = []
    for h in range(k // m):
        tabs.append(leaves(g[h * m:(h + 1) * m]))
    assert all(len(t) == 3 ** (m.bit_length() - 1) for t in tabs)
    rng = np.random.default_rng(k * 131 + m)
    cols = 24 if k <= 8 else 8
    data = rng.integers(0, 256, (k, cols), dtype=np.uint8)
    data[:, 0] = 0
    data[:, 1] = 255
    shards = np.zeros((1, k + m, cols), dtype=np.uint8)
    shards[0, :k] = data
    oracle.rs_encode(k, m, shards)
    for col in range(cols):
        y = [0] * m
        for h in range(k // m):
            part = conv(oracle, [int(v) for v in data[h * m:(h + 1) * m, col]], tabs[h])
            y = [a ^ b for a, b in zip(y, part)]
        assert y == [int(v) for v in shards[0, k:, col]], col


def test_non_power_of_two_codes_are_not_dyadic(oracle):
    """RS(20,10) (the reference's factory code) keeps the matrix form (no dyadic tables)."""
    M = oracle.build_matrix(20, 30)
    assert any(M[20 + i, j] != M[20, (i ^ j) % 20] for i in range(10) for j in range(20))
