"""BASELINE.json's configurations at their full batch sizes, through the C ABI, under -m gpu.

  #2 RS(2,3)   65 536 blocks, one erased data shard per block
  #3 RS(8,12)  2^20 blocks, one erased data shard per block (the bench workload)
  #4 RS(16,24) 2^19 blocks, U{1..8} losses uniform over all 24 shards
  RS(20,30)    2^19 blocks, U{1..10} losses uniform over all 30 shards (the reference's own code)

Each batch is generated on the device (include/fec_synth.h), encoded (fec_rs_encode_batch,
reed_solomon.go:51), recovered out of place (fec_rs_recover_batch, the device form of
recoverSymbolPayloads, reed_solomon.go:92-136) and rebuilt in place (fec_rs_reconstruct_batch,
ReconstructData, :124). Checked:
  * the whole batch round-trips: every rebuilt shard equals the erased original (a property
    that holds at any size, compared on the device);
  * 64 sampled blocks against the CPU oracle: their parity, and their recovered shards.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PAYLOAD, L, S = 1200, 1202, 1216
SEED = 0x0FEC


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU test needs a HIP device"
    return t


def _batch(torch, codec, k, m, B):
    data = torch.empty((B, k, S), dtype=torch.uint8, device="cuda")
    codec.synth_data(SEED, 0, B, k, PAYLOAD, data.data_ptr(), k * S, S)
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, 0)
    return data, par


def _sample_check(torch, oracle, k, m, data, par, lost, out, pick):
    """Sampled blocks: parity and recovered shards against the oracle (checker only)."""
    n = k + m
    d = data[pick].cpu().numpy()[:, :, :L]
    p = par[pick].cpu().numpy()[:, :, :L]
    sh = np.zeros((len(pick), n, L), dtype=np.uint8)
    sh[:, :k] = d
    oracle.rs_encode(k, m, sh)
    assert np.array_equal(p, sh[:, k:]), "parity of sampled blocks differs from the oracle"
    lo = lost[pick].cpu().numpy()
    masks = np.array([sum(1 << i for i in range(n) if not lo[j, i]) for j in range(len(pick))], dtype=np.uint32)
    dmg = sh.copy()
    dmg[lo] = 0x5A
    oracle.rs_reconstruct(k, m, dmg, masks)
    o = out[pick].cpu().numpy()[:, :, :L]
    for j in range(len(pick)):
        miss = [i for i in range(k) if lo[j, i]]
        for r, i in enumerate(miss):
            assert np.array_equal(o[j, r], dmg[j, i]), (int(pick[j]), r, i)


@pytest.mark.parametrize("k,m,B", [(2, 1, 65536), (8, 4, 1 << 20), (20, 10, 1 << 19)],
                         ids=["config2_rs2_3", "config3_rs8_12", "rs20_30_reference_code"])
def test_single_erasure_config_full_batch(fec, oracle, torch, k, m, B):
    codec = fec.Codec(0).use_torch_stream()
    try:
        n = k + m
        data, par = _batch(torch, codec, k, m, B)
        masks = torch.empty((B,), dtype=torch.int32, device="cuda")
        erased = torch.empty((B,), dtype=torch.int32, device="cuda")
        codec.synth_single_erasures(SEED, 0, B, k, m, masks.data_ptr(), erased.data_ptr())
        out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
        st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
        rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, masks.data_ptr(),
                                  out.data_ptr(), S, 1, st.data_ptr())
        assert rc == 0
        codec.sync()
        rows = torch.arange(B, device="cuda")
        er = erased.long()
        assert bool((st == 1).all())
        assert torch.equal(out[:, 0, :L], data[rows, er, :L]), "recovered shard != erased original"
        lost = torch.zeros((B, n), dtype=torch.bool, device="cuda")
        lost[rows, er] = True
        pick = np.sort(np.random.default_rng(k).choice(B, 64, replace=False))
        _sample_check(torch, oracle, k, m, data, par, lost, out, torch.from_numpy(pick).cuda())
        # in place: wipe every erased shard, rebuild, compare the whole batch
        want = data[rows, er].clone()
        data[rows, er] = 0
        rc = codec.rs_reconstruct_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S,
                                      masks.data_ptr(), None, fec.FEC_DEVICE)
        assert rc == 0
        codec.sync()
        assert torch.equal(data[rows, er, :L], want[:, :L])
    finally:
        codec.close()


@pytest.mark.parametrize("k,m", [(16, 8), (20, 10), (8, 4)], ids=["config4_rs16_24", "rs20_30_reference_code",
                                                                 "rs8_12_mixed"])
def test_mixed_erasures_full_batch(fec, oracle, torch, k, m):
    """2^19 blocks with e ~ U{1..m} lost shards per block, uniform over all n: RS(16,24) (config #4),
    RS(20,30), the reference's own sender/receiver code (manager.go:58-59,81-82), and RS(8,12)
    (the bench's code with multi-erasure blocks: the sorted-plan route with the runtime-k
    rebuild, which multi-slot calls of the small codes take since round 5)."""
    B = 1 << 19
    n = k + m
    codec = fec.Codec(0).use_torch_stream()
    try:
        data, par = _batch(torch, codec, k, m, B)
        g = torch.Generator(device="cuda")
        g.manual_seed({16: 0x1624, 20: 0x2030}.get(k, 0x0812))
        e = torch.randint(1, m + 1, (B,), device="cuda", generator=g)
        rank = torch.rand((B, n), device="cuda", generator=g).argsort(dim=1).argsort(dim=1)
        lost = rank < e[:, None]
        weights = torch.bitwise_left_shift(torch.ones(n, dtype=torch.int64, device="cuda"),
                                           torch.arange(n, device="cuda"))
        masks = ((~lost).to(torch.int64) * weights).sum(dim=1).to(torch.int32)
        e_d = lost[:, :k].sum(dim=1)
        slots = int(e_d.max().item())
        out = torch.zeros((B, slots, S), dtype=torch.uint8, device="cuda")
        st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
        rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S, masks.data_ptr(),
                                  out.data_ptr(), slots * S, slots, st.data_ptr())
        assert rc == 0
        codec.sync()
        assert torch.equal(st, e_d.to(torch.int32)), "status != erased data shards per block"
        # whole batch, out of place: slot r of block b holds its r-th lost data shard (ascending)
        order = torch.where(lost[:, :k], torch.arange(k, device="cuda"), k + torch.arange(k, device="cuda"))
        first = order.sort(dim=1).values[:, :slots]                    # lost data indices first, ascending
        for r in range(slots):
            sel = e_d > r
            idx = first[sel, r]
            rows = torch.nonzero(sel).squeeze(1)
            assert torch.equal(out[rows, r, :L], data[rows, idx, :L]), "recovered slot %d" % r
        pick = np.sort(np.random.default_rng(1624).choice(B, 64, replace=False))
        _sample_check(torch, oracle, k, m, data, par, lost, out, torch.from_numpy(pick).cuda())
        # in place over the whole batch
        want = data[:, :, :L].clone()
        data[lost[:, :k]] = 0
        rc = codec.rs_reconstruct_raw(k, m, L, B, data.data_ptr(), k * S, par.data_ptr(), m * S, S,
                                      masks.data_ptr(), None, fec.FEC_DEVICE)
        assert rc == 0
        codec.sync()
        assert torch.equal(data[:, :, :L], want)
    finally:
        codec.close()
