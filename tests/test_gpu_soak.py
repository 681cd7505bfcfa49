"""Seeded random soak of the batch codec against the CPU oracle (GPU; a complement to the
enumerated cases of test_gpu_codec.py).

Each case draws an RS code (k + m <= 32), a shard length on either side of every routing
threshold (16-byte chunks per shard: < 32 short-shard tile route, 32..63 wave route, >= 64 the
compile-time rebuilds; partial tail chunks), a batch size, a per-block loss count (up to m + 1, so
blocks with too few shards are mixed in) and a number of output slots (one: the direct
single-erasure kernel where the code has one; the largest data-loss count; or m), then checks
against the oracle (internal/fec reed_solomon.go:51,124 through klauspost's ReconstructData):
  * encode parity, bit-exact, pad bytes up to the 16-byte boundary written as zeros;
  * recover: per-block status (rebuilt count, -1 more erasures than slots, -4 too few shards)
    and every rebuilt shard, in ascending order of its index;
  * reconstruct in place: the data region of every block that has enough shards;
  * every fourth case also through the host-resident form (FEC_HOST, packed numpy shards).
XOR(k, 1) cases run beside them. The draws are fixed by the seed, so a failure names its case.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = 400
LENS = [1, 15, 16, 17, 200, 495, 496, 497, 512, 513, 1008, 1017, 1024, 1025, 1202, 1436]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU test needs a HIP device"
    return t


@pytest.fixture(scope="module")
def codec(fec):
    c = fec.Codec(0).use_torch_stream()
    yield c
    c.close()


def _draw(rng):
    if rng.random() < 0.15:
        k = int(rng.integers(1, 32))
        return "xor", k, 1
    n = int(rng.integers(2, 33))
    k = int(rng.integers(1, n))
    return "rs", k, n - k


def _masks(rng, B, n, max_loss):
    masks = np.empty(B, dtype=np.uint32)
    for b in range(B):
        e = int(rng.integers(0, max_loss + 1))
        lost = rng.choice(n, size=min(e, n), replace=False)
        masks[b] = ((1 << n) - 1) & ~int(sum(1 << int(i) for i in lost))
    return masks


@pytest.mark.parametrize("case", range(CASES))
def test_random_case_matches_oracle(codec, oracle, torch, fec, case):
    rng = np.random.default_rng(0x50AC + case)
    kind, k, m = _draw(rng)
    n = k + m
    L = int(rng.choice(LENS))
    S = (L + 15) // 16 * 16
    B = int(rng.choice([1, 3, 64, 65, 300]))
    sh = np.zeros((B, n, S), dtype=np.uint8)
    sh[:, :k, :L] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    ref = sh.copy()
    if kind == "xor":
        oracle.xor_encode(k, ref)
    else:
        oracle.rs_encode(k, m, ref)
    ref[:, k:, L:] = 0
    sh[:, k:] = 0xA5   # parity slots pre-filled: the pad bytes must come back as zeros
    d = torch.from_numpy(sh).cuda()
    if kind == "xor":
        codec.xor_encode(k, d, shard_len=L)
    else:
        codec.rs_encode(k, m, d, shard_len=L)
    codec.sync()
    got = d.cpu().numpy()
    assert np.array_equal(got[:, k:], ref[:, k:]), (kind, k, m, L, B, "parity")

    masks = _masks(rng, B, n, min(n, m + 1))
    lost = ~((masks[:, None] >> np.arange(n)[None, :]) & 1).astype(bool)
    e_d = lost[:, :k].sum(axis=1)
    few = (n - lost.sum(axis=1)) < k
    dm = torch.from_numpy(masks.view(np.int32)).cuda()

    if kind == "xor":
        dmg = ref.copy()
        dmg[:, :k][lost[:, :k]] = 0xC3
        dd = torch.from_numpy(dmg).cuda()
        st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
        codec.xor_reconstruct(k, dd, dm, status=st, shard_len=L)
        rc = codec.lib_sync_rc()
        bad = (e_d > 0) & few
        assert rc == (fec.FEC_ERR_TOO_FEW_SHARDS if bad.any() else fec.FEC_OK)
        s = st.cpu().numpy()
        assert np.array_equal(s, np.where(bad, -4, 0)), (kind, k, L, B, "status")
        g = dd.cpu().numpy()
        ok = ~bad
        assert np.array_equal(g[ok, :k, :L], ref[ok, :k, :L]), (kind, k, L, B, "rebuilt")
        return

    # recover into one slot, the largest data-loss count, or m slots
    slots = int(rng.choice([1, max(1, int(e_d.max())), m]))
    want_st = np.where(e_d == 0, 0, np.where(few, -4, np.where(e_d > slots, -1, e_d)))
    data = torch.from_numpy(np.ascontiguousarray(ref[:, :k])).cuda()
    data[torch.from_numpy(lost[:, :k]).cuda()] = 0x3C
    par = torch.from_numpy(np.ascontiguousarray(ref[:, k:])).cuda()
    out = torch.full((B, slots, S), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    codec.rs_recover_split(k, m, data, par, dm, out, status=st, shard_len=L)
    if (want_st < 0).any():
        with pytest.raises(fec.FecError):
            codec.sync()
    else:
        codec.sync()
    tag = (k, m, L, B, slots)
    assert np.array_equal(st.cpu().numpy(), want_st), (tag, "status")
    o = out.cpu().numpy()
    for b in np.nonzero(want_st > 0)[0]:
        for r, i in enumerate(np.nonzero(lost[b, :k])[0]):
            assert np.array_equal(o[b, r, :L], ref[b, i, :L]), (tag, int(b), r, int(i))
    # in place: every block with enough shards comes back whole
    codec.rs_reconstruct_split(k, m, data, par, dm, shard_len=L)
    if few.any() and (e_d[few] > 0).any():
        with pytest.raises(fec.FecError):
            codec.sync()
    else:
        codec.sync()
    g = data.cpu().numpy()
    ok = ~few | (e_d == 0)
    assert np.array_equal(g[ok, :, :L], ref[ok, :k, :L]), (tag, "in place")
    if case % 4 == 0:
        # the host-resident form (FEC_HOST: numpy buffers staged through pinned memory), packed
        # shards (stride = shard length) as the reference's per-block slices are
        hs = np.ascontiguousarray(ref[:, :, :L])
        enc = hs.copy()
        enc[:, k:] = 0
        codec.rs_encode(k, m, enc)
        assert np.array_equal(enc, hs), (tag, "host parity")
        dmg = hs.copy()
        dmg[lost] = 0x77
        hst = np.full(B, 7, dtype=np.int32)
        rc = codec.rs_reconstruct(k, m, dmg, masks, status=hst)
        bad = few & (e_d > 0)
        assert rc == (fec.FEC_ERR_TOO_FEW_SHARDS if bad.any() else fec.FEC_OK), (tag, "host rc")
        assert np.array_equal(hst == 0, ~bad), (tag, "host status")
        assert np.array_equal(dmg[~bad, :k], hs[~bad, :k]), (tag, "host rebuilt")
