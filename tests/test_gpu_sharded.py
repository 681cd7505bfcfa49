"""BASELINE config #5 on one GPU: RS(8,12) over a global batch sharded across 8 ranks
(independent per-GPU block ranges, no collective on the data path).

The 8 ranks run in sequence through bench.py's own per-rank code (shard.block_range, the
rank's slice of the device-generated global batch, RankStep encode + recover) on one device.
Every rank's bytes are checked against the host restatement of the generator and the CPU
oracle, and the union of the ranks' parity equals one pass over the whole batch."""
import importlib
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU test needs a HIP device"
    return t


@pytest.fixture(scope="module")
def bench():
    sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


@pytest.fixture(scope="module")
def shard(fec):
    return importlib.import_module("0xfec_amd.shard")


@pytest.mark.parametrize("payload,stride", [(1200, 1216), (1, 16), (17, 32), (1434, 1440), (1201, 1216)])
def test_device_generator_equals_host_restatement(fec, torch, shard, payload, stride):
    codec = fec.Codec(0).use_torch_stream()
    k, m, lo, nb = 5, 3, 123457, 37
    d = torch.full((nb, k, stride), 0xEE, dtype=torch.uint8, device="cuda")
    codec.synth_data(0x0FEC, lo, nb, k, payload, d.data_ptr(), k * stride, stride)
    masks = torch.empty(nb, dtype=torch.int32, device="cuda")
    er = torch.empty(nb, dtype=torch.int32, device="cuda")
    codec.synth_single_erasures(0x0FEC, lo, nb, k, m, masks.data_ptr(), er.data_ptr())
    codec.sync()
    assert np.array_equal(d.cpu().numpy(), shard.synth_payload_blocks(0x0FEC, lo, lo + nb, k, payload, stride))
    want_e = shard.synth_single_erasures(0x0FEC, lo, lo + nb, k)
    assert np.array_equal(er.cpu().numpy(), want_e)
    assert np.array_equal(masks.cpu().numpy().view(np.uint32), ((1 << (k + m)) - 1) & ~(1 << want_e).astype(np.uint32))
    codec.close()


def test_eight_ranks_in_sequence_equal_one_pass(fec, torch, shard, bench, oracle):
    k, m, world, per_rank = 8, 4, 8, 2500
    total = world * per_rank + 3                 # ragged: ranks differ by one block
    seed = 0x0FEC
    codec = fec.Codec(0)
    codec.prepare(k, m)
    codec.use_torch_stream()
    dev = torch.device("cuda", 0)
    parts = []
    for rank in range(world):
        lo, hi = shard.block_range(total, rank, world)
        b = bench.RankBatch(torch, codec, dev, hi - lo, k, m, seed, lo)
        st = bench.RankStep(fec, codec, b)
        st.encode()
        st.decode()
        codec.sync()
        data = b.data.cpu().numpy()
        assert np.array_equal(data, shard.synth_payload_blocks(seed, lo, hi, k, bench.PAYLOAD, bench.SHARD_STRIDE))
        er = b.erased.cpu().numpy()
        assert np.array_equal(er, shard.synth_single_erasures(seed, lo, hi, k))
        # every block's recovered shard is its erased data shard
        rec = b.recovered.cpu().numpy()[:, 0, :bench.SHARD_LEN]
        assert np.array_equal(rec, data[np.arange(hi - lo), er, :bench.SHARD_LEN])
        # sampled blocks of this rank against the CPU oracle (encode)
        pick = np.random.default_rng(rank).choice(hi - lo, 48, replace=False)
        sh = np.zeros((48, k + m, bench.SHARD_LEN), dtype=np.uint8)
        sh[:, :k] = data[pick, :, :bench.SHARD_LEN]
        oracle.rs_encode(k, m, sh)
        assert np.array_equal(b.parity.cpu().numpy()[pick, :, :bench.SHARD_LEN], sh[:, k:])
        assert st.check_full(torch)
        parts.append(b.parity.cpu().numpy())
        del b, st
    whole = bench.RankBatch(torch, codec, dev, total, k, m, seed, 0)
    bench.RankStep(fec, codec, whole).encode()
    codec.sync()
    assert np.array_equal(np.concatenate(parts), whole.parity.cpu().numpy())
    codec.close()
