"""The SIMD restatement of klauspost's kernels (oracle/fec_simd.c: AVX2 nibble PSHUFB,
GFNI-AVX2 and GFNI-AVX-512 affine forms), used as bench.py's cpu_baseline, is bit-exact against
the scalar oracle (fec_oracle.c, pinned to the reference's golden vectors) for encode and
ReconstructData: shapes of the reference (RS(20,10)), the bench (RS(2,3), RS(8,12), RS(16,24))
and odd ones, shard lengths with and without a vector tail, random erasure patterns. ISAs the
host lacks are skipped."""
import numpy as np
import pytest


def _isas(oracle):
    return [i for i in (oracle.ISA_SCALAR, oracle.ISA_AVX2, oracle.ISA_GFNI_AVX2, oracle.ISA_GFNI_AVX512)
            if oracle.isa_supported(i)]


@pytest.mark.parametrize("k,m", [(2, 1), (6, 2), (8, 4), (16, 8), (20, 10), (5, 27)])
@pytest.mark.parametrize("L", [1, 31, 64, 100, 1202, 1436])
def test_simd_encode_matches_scalar(oracle, k, m, L):
    rng = np.random.default_rng(k * 1000 + L)
    B, n = 9, k + m
    sh = np.zeros((B, n, L), dtype=np.uint8)
    sh[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    want = oracle.rs_encode(k, m, sh.copy())
    for isa in _isas(oracle):
        got = sh.copy()
        got[:, k:] = 0x5A
        oracle.rs_encode_simd(k, m, got, isa)
        assert np.array_equal(got, want), oracle.isa_name(isa)


@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8), (20, 10)])
@pytest.mark.parametrize("L", [33, 1202])
def test_simd_reconstruct_matches_scalar(oracle, k, m, L):
    rng = np.random.default_rng(k * 77 + L)
    B, n = 64, k + m
    sh = np.zeros((B, n, L), dtype=np.uint8)
    sh[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    oracle.rs_encode(k, m, sh)
    masks = np.empty(B, dtype=np.uint32)
    for b in range(B):
        lost = rng.choice(n, size=int(rng.integers(0, m + 2)), replace=False)   # some blocks unrecoverable
        masks[b] = ((1 << n) - 1) & ~int(sum(1 << int(i) for i in lost))
    wiped = sh.copy()
    for b in range(B):
        for i in range(k):
            if not masks[b] >> i & 1:
                wiped[b, i] = 0xC3
    want = wiped.copy()
    st_want = oracle.rs_reconstruct(k, m, want, masks)
    for isa in _isas(oracle):
        got = wiped.copy()
        st = oracle.rs_reconstruct_simd(k, m, got, masks, isa)
        assert np.array_equal(st, st_want) and np.array_equal(got, want), oracle.isa_name(isa)
    ok = st_want == 0
    assert np.array_equal(want[ok, :k], sh[ok, :k])


def test_best_isa_is_supported(oracle):
    assert oracle.isa_supported(oracle.best_isa())
