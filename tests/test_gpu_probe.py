"""The traffic twins of include/fec_probe.h move the bytes their kernels move: the encode twin
reads all k data shards of every block and writes all m output shards (output r = XOR of inputs
j with j % m == r, bytes past the shard length zero), the recover twin reads exactly the k-1
other data shards and the first present parity of each single-erasure block and writes their XOR
to the block's output slot (other blocks untouched), and the rebuild twin reads the first k present
shards of each block and writes their XOR into one output row per erased data shard. Checked against numpy on the same bytes, so
a twin that skipped or re-read shards would show up here before it skewed a bench line."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

S, L = 1216, 1202


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU test needs a HIP device"
    return t


@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8), (20, 10)])
def test_encode_twin_reads_and_writes_every_shard(fec, torch, k, m):
    codec = fec.Codec(0)
    B = 777
    rng = np.random.default_rng(k)
    host = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    data = torch.from_numpy(host).cuda()
    par = torch.full((B, m, S), 0xAB, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    codec.probe_encode_traffic_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S)
    codec.sync()
    want = np.zeros((B, m, S), dtype=np.uint8)
    for j in range(k):
        want[:, j % m] ^= host[:, j]
    want[:, :, L:] = 0
    assert np.array_equal(par.cpu().numpy(), want)
    codec.close()


@pytest.mark.parametrize("k,m", [(8, 4), (20, 10)])
def test_recover_twin_reads_the_decode_inputs(fec, torch, k, m):
    codec = fec.Codec(0)
    B = 501
    rng = np.random.default_rng(100 + k)
    dh = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    ph = rng.integers(0, 256, (B, m, S), dtype=np.uint8)
    n = k + m
    masks = np.full(B, (1 << n) - 1, dtype=np.uint32)
    erased = rng.integers(0, k, B)
    lostp = rng.integers(0, m, B)
    for b in range(B):
        masks[b] &= ~np.uint32(1 << int(erased[b]))
        if b % 3 == 0:
            masks[b] &= ~np.uint32(1 << (k + int(lostp[b])))   # a later parity is the first present
    masks[7] &= ~np.uint32(3)          # two data erasures: not a single-erasure block
    data, par = torch.from_numpy(dh).cuda(), torch.from_numpy(ph).cuda()
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    out = torch.full((B, 1, S), 0xCD, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    codec.probe_recover_traffic_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, dm.data_ptr(),
                                    out.data_ptr(), S)
    codec.sync()
    got = out.cpu().numpy()[:, 0]
    for b in range(B):
        mk = int(masks[b])
        if b == 7:
            assert (got[b] == 0xCD).all()
            continue
        r0 = next(r for r in range(m) if mk >> (k + r) & 1)
        w = ph[b, r0].copy()
        for j in range(k):
            if j != erased[b]:
                w ^= dh[b, j]
        w[L:] = 0
        assert np.array_equal(got[b], w), b
    codec.close()


@pytest.mark.parametrize("k,m", [(16, 8), (20, 10)])
def test_rebuild_twin_reads_the_first_k_present(fec, torch, k, m):
    codec = fec.Codec(0)
    B = 613
    n = k + m
    rng = np.random.default_rng(300 + k)
    dh = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    ph = rng.integers(0, 256, (B, m, S), dtype=np.uint8)
    masks = np.empty(B, dtype=np.uint32)
    for b in range(B):
        lost = rng.choice(n, size=int(rng.integers(0, m + 1)), replace=False)
        masks[b] = ((1 << n) - 1) & ~int(sum(1 << int(i) for i in lost))
    masks[5] = ((1 << n) - 1) & ~((1 << (m + 1)) - 1)   # m + 1 losses: unrecoverable, nothing moved
    data, par = torch.from_numpy(dh).cuda(), torch.from_numpy(ph).cuda()
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    out = torch.full((B, m, S), 0xCD, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    codec.probe_rebuild_traffic_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, dm.data_ptr(),
                                    out.data_ptr(), m * S)
    codec.sync()
    got = out.cpu().numpy()
    for b in range(B):
        mk = int(masks[b])
        present = [i for i in range(n) if mk >> i & 1]
        e = sum(1 for i in range(k) if not mk >> i & 1)
        if e == 0 or len(present) < k:
            assert (got[b] == 0xCD).all(), b
            continue
        w = np.zeros(S, dtype=np.uint8)
        for i in present[:k]:
            w ^= dh[b, i] if i < k else ph[b, i - k]
        w[L:] = 0
        for r in range(m):
            assert np.array_equal(got[b, r], w) if r < e else (got[b, r] == 0xCD).all(), (b, r)
    codec.close()
