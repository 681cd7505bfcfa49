"""GPU parity of the batch codec (C ABI, include/fec_hip.h) against the CPU oracle.

Bit-exact comparison on seeded inputs, device-resident (FEC_DEVICE via torch CUDA tensors) and
host-resident (FEC_HOST via numpy), over shapes that cover the reference's configurations
(XOR(2,1), RS(6,2), RS(20,10) factories and tests: internal/fec/manager.go:54-90,
reed_solomon_test.go) and the benchmark ones (RS(2,3)-style (2,1), (8,4), (16,8)),
odd shard lengths (tail chunks), every erasure count, and the too-few-shards error.
"""
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = [(1, 1), (2, 1), (3, 2), (6, 2), (8, 4), (16, 8), (20, 10), (5, 11), (31, 1), (10, 22)]
LENS = [1, 2, 3, 15, 16, 17, 33, 1202, 1436]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU test needs a HIP device"
    return t


@pytest.fixture(scope="module")
def codec(fec):
    import torch
    c = fec.Codec(0).use_torch_stream()
    yield c
    c.close()


def _rand_shards(rng, B, n, S, L):
    sh = np.zeros((B, n, S), dtype=np.uint8)
    sh[:, :, :L] = rng.integers(0, 256, (B, n, L), dtype=np.uint8)
    return sh


def _random_masks(rng, B, k, m, max_loss=None):
    n = k + m
    max_loss = m if max_loss is None else max_loss
    masks = np.empty(B, dtype=np.uint32)
    for b in range(B):
        e = int(rng.integers(0, max_loss + 1))
        lost = rng.choice(n, size=e, replace=False)
        masks[b] = ((1 << n) - 1) & ~int(sum(1 << int(i) for i in lost))
    return masks


@pytest.mark.parametrize("k,m", SHAPES)
@pytest.mark.parametrize("L", LENS)
def test_rs_encode_device_matches_oracle(codec, oracle, torch, k, m, L):
    rng = np.random.default_rng(1000 * k + 10 * m + L)
    n = k + m
    S = (L + 15) // 16 * 16 + 16 * int(rng.integers(0, 2))
    B = 37
    sh = _rand_shards(rng, B, n, S, L)
    sh[:, k:, :] = 0xA5                          # parity slots pre-filled
    ref = sh.copy()
    oracle.rs_encode(k, m, ref)
    ref[:, k:, L:] = 0xA5                        # past the 16-byte boundary: untouched
    ref[:, k:, L:(L + 15) // 16 * 16] = 0        # up to it: zero padding (fec_hip.h)
    d = torch.from_numpy(sh).cuda()
    codec.rs_encode(k, m, d, shard_len=L)
    codec.sync()
    got = d.cpu().numpy()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("k,m", SHAPES)
@pytest.mark.parametrize("L", [1, 17, 1202])
def test_rs_reconstruct_device_matches_oracle(codec, oracle, torch, k, m, L):
    if k + m > 32:
        pytest.skip("decode limited to n <= 32")
    rng = np.random.default_rng(7 * k + m + L)
    n = k + m
    S = (L + 15) // 16 * 16
    B = 301
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = _random_masks(rng, B, k, m, max_loss=min(n, m + 1))
    damaged = sh.copy()
    for b in range(B):
        for i in range(n):
            if not (masks[b] >> i) & 1:
                damaged[b, i, :] = 0x5A
    ref = damaged.copy()
    st_ref = oracle.rs_reconstruct(k, m, ref, masks, length=L)
    d = torch.from_numpy(damaged).cuda()
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    ds = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    codec.rs_reconstruct(k, m, d, dm, status=ds, shard_len=L)
    st = ds.cpu().numpy()
    assert np.array_equal(st == 0, st_ref == 0)
    assert set(np.unique(st)).issubset({0, -4})
    got = d.cpu().numpy()
    # rebuilt shards carry zero padding up to the 16-byte boundary of their slot
    for b in range(B):
        if st_ref[b] == 0:
            for i in range(k):
                if not (masks[b] >> i) & 1:
                    ref[b, i, L:(L + 15) // 16 * 16] = 0
    assert np.array_equal(got, ref)
    # recovered blocks equal the original data
    ok = st_ref == 0
    assert np.array_equal(got[ok, :k, :L], sh[ok, :k, :L])
    if (st_ref != 0).any():
        from importlib import import_module
        fec = import_module("0xfec_amd")
        with pytest.raises(fec.FecError):
            codec.sync()
    else:
        codec.sync()


def test_rs_every_erasure_pattern_8_12(codec, oracle, torch):
    """Every pattern of <= 4 losses of RS(8,12) (794 patterns), 1202-byte shards."""
    k, m, L = 8, 4, 1202
    n = k + m
    pats = [p for r in range(0, m + 1) for p in itertools.combinations(range(n), r)]
    B = len(pats)
    rng = np.random.default_rng(0x0FEC)
    S = 1216
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = np.array([((1 << n) - 1) & ~sum(1 << i for i in p) for p in pats], dtype=np.uint32)
    dmg = sh.copy()
    for b, p in enumerate(pats):
        for i in p:
            dmg[b, i] = 0
    d = torch.from_numpy(dmg).cuda()
    codec.rs_reconstruct(k, m, d, torch.from_numpy(masks.view(np.int32)).cuda())
    codec.sync()
    got = d.cpu().numpy()
    assert np.array_equal(got[:, :k, :L], sh[:, :k, :L])


@pytest.mark.parametrize("k,m", [(2, 1), (6, 2), (8, 4), (20, 10)])
def test_rs_host_path_matches_oracle(codec, oracle, k, m):
    fec = __import__("importlib").import_module("0xfec_amd")
    rng = np.random.default_rng(k * m)
    n, L = k + m, 1202
    B = 129
    sh = _rand_shards(rng, B, n, L, L)       # packed host layout, stride == shard_len
    ref = sh.copy()
    oracle.rs_encode(k, m, ref)
    codec.rs_encode(k, m, sh)
    assert np.array_equal(sh, ref)
    masks = _random_masks(rng, B, k, m)
    dmg = sh.copy()
    for b in range(B):
        for i in range(n):
            if not (masks[b] >> i) & 1:
                dmg[b, i] = 0
    st = np.full(B, 7, dtype=np.int32)
    rc = codec.rs_reconstruct(k, m, dmg, masks, status=st)
    assert rc == fec.FEC_OK and (st == 0).all()
    assert np.array_equal(dmg[:, :k], sh[:, :k])


@pytest.mark.parametrize("wpc", [6, 0])
@pytest.mark.parametrize("k", [1, 2, 3, 5, 9, 31])
@pytest.mark.parametrize("L", [1, 6, 18, 513, 1202, 1436])
def test_xor_device_matches_oracle(codec, oracle, torch, fec, tune, wpc, k, L):
    # L = 513: 33 chunks per shard, so a wave's 64 items span three blocks (the reconstruct's
    # scalar mask loads take up to three); L < 497: the per-lane mask load. wpc: the shipped
    # residency of both XOR kernels (6 workgroups/CU) and as many as fit
    tune(xor_wpc=wpc)
    rng = np.random.default_rng(k + L)
    n = k + 1
    S = (L + 15) // 16 * 16
    B = 65
    sh = _rand_shards(rng, B, n, S, L)
    ref = sh.copy()
    oracle.xor_encode(k, ref)
    d = torch.from_numpy(sh).cuda()
    codec.xor_encode(k, d, shard_len=L)
    codec.sync()
    enc = d.cpu().numpy()
    assert np.array_equal(enc[:, :, :L], ref[:, :, :L])
    masks = _random_masks(rng, B, k, 1, max_loss=2)
    dmg = enc.copy()
    for b in range(B):
        for i in range(n):
            if not (masks[b] >> i) & 1:
                dmg[b, i] = 0x33
    want = dmg.copy()
    st_ref = oracle.xor_reconstruct(k, want, masks)
    dd = torch.from_numpy(dmg).cuda()
    ds = torch.zeros(B, dtype=torch.int32, device="cuda")
    codec.xor_reconstruct(k, dd, torch.from_numpy(masks.view(np.int32)).cuda(), status=ds, shard_len=L)
    rc = codec.lib_sync_rc()
    assert rc == (fec.FEC_ERR_TOO_FEW_SHARDS if (st_ref != 0).any() else fec.FEC_OK)
    got = dd.cpu().numpy()
    st = ds.cpu().numpy()
    assert np.array_equal(st == 0, st_ref == 0)
    ok = st_ref == 0
    assert np.array_equal(got[ok][:, :, :L], want[ok][:, :, :L])


def test_argument_errors(codec, torch, fec):
    d = torch.zeros((4, 3, 32), dtype=torch.uint8, device="cuda")
    with pytest.raises(fec.FecError) as e:
        codec.rs_encode(0, 3, d)
    assert e.value.code == fec.FEC_ERR_INV_SHARD_NUM
    with pytest.raises(fec.FecError) as e:
        codec.rs_encode_raw(200, 57, 16, 1, d.data_ptr(), 32, d.data_ptr(), 32, 16, fec.FEC_DEVICE)
    assert e.value.code == fec.FEC_ERR_MAX_SHARD_NUM
    with pytest.raises(fec.FecError) as e:
        codec.rs_encode_raw(2, 1, 16, 1, d.data_ptr() + 1, 48, d.data_ptr() + 33, 48, 16, fec.FEC_DEVICE)
    assert e.value.code == fec.FEC_ERR_ALIGNMENT
    with pytest.raises(fec.FecError) as e:
        codec.rs_encode_raw(2, 1, 0, 1, d.data_ptr(), 48, d.data_ptr() + 32, 48, 16, fec.FEC_DEVICE)
    assert e.value.code == fec.FEC_ERR_SHARD_NO_DATA
    assert codec.rs_reconstruct_raw(20, 13, 16, 1, d.data_ptr(), 48, d.data_ptr(), 48, 16, d.data_ptr(), None,
                                    fec.FEC_DEVICE) == fec.FEC_ERR_MAX_SHARD_NUM
    # empty batches are no-ops
    codec.rs_encode_raw(2, 1, 16, 0, d.data_ptr(), 48, d.data_ptr() + 32, 48, 16, fec.FEC_DEVICE)
    codec.sync()


# FEC_DEVICE masks and statuses are read and written as 4-byte words (the kernels read the masks by
# scalar loads, which drop the low two address bits): every reconstruct / recover entry point
# refuses a mask or status array that is not 4-byte aligned (fec_hip.h), on every route, before
# anything is enqueued.
@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8)])
def test_misaligned_masks_and_status_refused(codec, torch, fec, k, m):
    B, S, L = 8, 1216, 1202
    n = k + m
    sh = torch.zeros((B, n, S), dtype=torch.uint8, device="cuda")
    mk = torch.zeros(B + 2, dtype=torch.int32, device="cuda")
    st = torch.zeros(B + 2, dtype=torch.int32, device="cuda")
    out = torch.zeros((B, 1, S), dtype=torch.uint8, device="cuda")
    d, p = sh.data_ptr(), sh.data_ptr() + k * S
    for ma, sa in ((mk.data_ptr() + 2, None), (mk.data_ptr(), st.data_ptr() + 1)):
        assert codec.rs_reconstruct_raw(k, m, L, B, d, n * S, p, n * S, S, ma, sa, fec.FEC_DEVICE) == \
            fec.FEC_ERR_ALIGNMENT
        assert codec.rs_recover_raw(k, m, L, B, d, n * S, p, n * S, S, ma, out.data_ptr(), S, 1, sa) == \
            fec.FEC_ERR_ALIGNMENT
    assert fec.lib.fec_xor_reconstruct_batch(codec.handle, 2, L, B, d, 3 * S, d + 2 * S, 3 * S, S,
                                             mk.data_ptr() + 1, None, fec.FEC_DEVICE) == fec.FEC_ERR_ALIGNMENT
    codec.sync()


# In-place RS(8,12) reconstructs take the routed form (fec_recover.hip): a classify pass, then the
# direct single-erasure body when no recoverable block has two or more erased data shards, else the
# sorted plans and the wave rebuild. Batches on either side of that line, with intact blocks,
# parity-only losses and too-few-shards blocks mixed in, sizes around the classify pass's 256-block
# sweep and the 64-block plan windows, against the oracle (data and statuses), on the routed form
# on round 5's sorted-plan route (dec_route 0), and on the routed form whose direct route runs all
# four waves of each workgroup (route_ww 4; the default runs three over a larger grid, the plan
# route on its first total / 256 workgroups).
ROUTE_FORMS = {0: dict(dec_route=0), 1: dict(dec_route=1), 2: dict(dec_route=1, route_ww=4)}


@pytest.mark.parametrize("route", [1, 0, 2])
@pytest.mark.parametrize("B", [1, 63, 257, 1031])
@pytest.mark.parametrize("multi", [False, True])
def test_rs_inplace_routed_matches_oracle(codec, oracle, torch, fec, tune, route, B, multi):
    k, m, L, S = 8, 4, 1202, 1216
    n = k + m
    rng = np.random.default_rng(B * 7 + int(multi) + 10 * route)
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = np.empty(B, dtype=np.uint32)
    for b in range(B):
        kind = int(rng.integers(0, 5))
        if kind == 0:
            lost = []                                                      # intact
        elif kind == 1:
            lost = [int(rng.integers(k, n))]                               # one parity shard
        elif kind == 2 or (kind == 3 and not multi):
            lost = [int(rng.integers(0, k))]                               # one data shard
        elif kind == 3:
            lost = list(rng.choice(n, size=int(rng.integers(2, m + 1)), replace=False))   # up to m shards
        else:
            lost = list(rng.choice(k, size=m + 1, replace=False))          # too few shards
        masks[b] = ((1 << n) - 1) & ~sum(1 << int(i) for i in lost)
    if multi:   # at least one block with two erased data shards (the plan route)
        masks[B // 2] = ((1 << n) - 1) & ~0b101
    dmg = sh.copy()
    for b in range(B):
        for i in range(n):
            if not (masks[b] >> i) & 1:
                dmg[b, i] = 0x3C
    want = dmg.copy()
    st_ref = oracle.rs_reconstruct(k, m, want, masks, length=L)
    tune(**ROUTE_FORMS[route])
    d = torch.from_numpy(np.ascontiguousarray(dmg[:, :k])).cuda()
    par = torch.from_numpy(np.ascontiguousarray(dmg[:, k:])).cuda()
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    codec.rs_reconstruct_split(k, m, d, par, torch.from_numpy(masks.view(np.int32)).cuda(), status=st,
                               shard_len=L)
    rc = codec.lib_sync_rc()
    assert rc == (fec.FEC_ERR_TOO_FEW_SHARDS if (st_ref != 0).any() else fec.FEC_OK)
    assert np.array_equal(st.cpu().numpy() == 0, st_ref == 0)
    got = d.cpu().numpy()
    ok = st_ref == 0
    assert np.array_equal(got[ok][:, :, :L], sh[ok][:, :k, :L])


@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8), (20, 10)])
def test_rs_split_layout_matches_interleaved(codec, oracle, torch, k, m):
    """Data and parity in separate buffers (the bench layout) give the same bytes."""
    rng = np.random.default_rng(99 + k)
    n, L, S, B = k + m, 1202, 1216, 203
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    data = torch.from_numpy(np.ascontiguousarray(sh[:, :k])).cuda()
    par = torch.zeros((B, m, S), dtype=torch.uint8, device="cuda")
    codec.rs_encode_split(k, m, data, par, shard_len=L)
    codec.sync()
    assert np.array_equal(par.cpu().numpy()[:, :, :L], sh[:, k:, :L])
    masks = _random_masks(rng, B, k, m)
    want = sh.copy()
    for b in range(B):
        for i in range(k):
            if not (masks[b] >> i) & 1:
                data[b, i] = 0x77
    st = torch.zeros(B, dtype=torch.int32, device="cuda")
    codec.rs_reconstruct_split(k, m, data, par, torch.from_numpy(masks.view(np.int32)).cuda(), status=st,
                               shard_len=L)
    codec.sync()
    assert (st.cpu().numpy() == 0).all()
    assert np.array_equal(data.cpu().numpy()[:, :, :L], want[:, :k, :L])


@pytest.mark.parametrize("k,m,slots", [(8, 4, 1), (8, 4, 4), (16, 8, 8), (20, 10, 3)])
def test_rs_recover_out_of_place(codec, oracle, torch, fec, k, m, slots):
    """fec_rs_recover_batch writes the erased data shards, ascending, to a separate buffer
    (the shape of recoverSymbolPayloads' result) and leaves the inputs untouched."""
    rng = np.random.default_rng(7 * k + slots)
    n, L, S, B = k + m, 1202, 1216, 257
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = _random_masks(rng, B, k, m)
    data_np = np.ascontiguousarray(sh[:, :k]).copy()
    for b in range(B):
        for i in range(k):
            if not (masks[b] >> i) & 1:
                data_np[b, i] = 0x11
    data = torch.from_numpy(data_np).cuda()
    par = torch.from_numpy(np.ascontiguousarray(sh[:, k:])).cuda()
    out = torch.full((B, slots, S), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    codec.rs_recover_split(k, m, data, par, torch.from_numpy(masks.view(np.int32)).cuda(), out, status=st,
                           shard_len=L)
    over = False
    try:
        codec.sync()
    except fec.FecError as e:
        assert e.code == fec.FEC_ERR_INVALID_ARG
        over = True
    st = st.cpu().numpy()
    got = out.cpu().numpy()
    assert np.array_equal(data.cpu().numpy(), data_np)          # inputs untouched
    saw_over = False
    for b in range(B):
        miss = [i for i in range(k) if not (masks[b] >> i) & 1]
        if len(miss) > slots:
            assert st[b] == fec.FEC_ERR_INVALID_ARG
            saw_over = True
            continue
        assert st[b] == len(miss)
        for r, i in enumerate(miss):
            assert np.array_equal(got[b, r, :L], sh[b, i, :L])
    assert saw_over == over


# Every shipped RS encode kernel against the oracle: the code's own kernel (RS(2,3) by its parity
# row, RS(8,12) dyadic, RS(16,24) / RS(20,30) bit-sliced; every other shape the generic kernel) and
# the generic kernel on the reference's shapes too (knob enc_fixed 0), at residency caps of the
# fixed-shape forms, over batch sizes and tails that leave workgroups empty, partial and ragged.
ENC_VARIANTS = {
    "own": dict(enc_fixed=1),
    "own_wpc2": dict(enc_fixed=1, enc_wpc=2, enc_bwpc=2),
    "generic": dict(enc_fixed=0),
    "generic_wpc2": dict(enc_fixed=0, gen_wpc=2),
    "stpol_nt": dict(enc_fixed=1, st_pol=0),
    "ww2_wpc4": dict(enc_fixed=1, enc_ww=2, enc_wpc=4),
    "ww4": dict(enc_fixed=1, enc_ww=4),
}


@pytest.mark.parametrize("variant", sorted(ENC_VARIANTS))
@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8), (20, 10)])
@pytest.mark.parametrize("B,L", [(1, 1), (3, 17), (37, 1202), (1000, 1202), (4099, 1436), (20000, 33)])
def test_rs_encode_kernel_variants_match_oracle(codec, oracle, torch, variant, k, m, B, L):
    rng = np.random.default_rng(B * 31 + L * 7 + k)
    n = k + m
    S = (L + 15) // 16 * 16
    data = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    data[:, :, L:] = 0
    ref = np.zeros((B, n, S), dtype=np.uint8)
    ref[:, :k] = data
    oracle.rs_encode(k, m, ref)
    d = torch.from_numpy(data).cuda()
    p = torch.full((B, m, S), 0xA5, dtype=torch.uint8, device="cuda")
    old = codec.set_tuning(**ENC_VARIANTS[variant])
    try:
        codec.rs_encode_split(k, m, d, p, shard_len=L)
        codec.sync()
    finally:
        codec.set_tuning(**old)
    got = p.cpu().numpy()
    assert np.array_equal(got[:, :, :L], ref[:, k:, :L])
    assert not got[:, :, L:].any()               # pad to the 16-byte boundary written as zeros


# Every shipped reconstruct path against the oracle, in place and out of place (m slots), with the
# erasure counts mixed inside waves: "default" (the direct kernel for RS(2,3) and the other m = 1
# codes; sorted plans + the rebuild for the rest: fec_rebuild.hip for RS(16,24) / RS(20,30) where
# shards have 64+ chunks, the compile-time-k or runtime-k wave form below that), "plan" (no direct
# kernel: sorted plans + the wave form for every code), "tile" (plans in block order + the
# workgroup-tile rebuild, the short-shard path, on long shards too), "table" (the direct kernel's
# rows copied from the PermTab table rather than expanded from the kernel argument), and "wpc2"
# (the default at two workgroups per CU). L = 1008 / 1017: shards of 63 / 64 chunks, the edge of
# the rebuild's two-block slices. The single-slot test below covers the direct kernel of the
# m >= 2 codes.
DEC_VARIANTS = {
    "default": {},
    "plan": dict(dec_direct=0),
    "tile": dict(dec_direct=0, dec_wave=0),
    "table": dict(dec_direct=2),
    "wpc2": dict(dir_wpc=2, dec_wpc=2),
    "noroute": dict(dec_route=0),
    "dstpol_nt": dict(dst_pol=0),
}


@pytest.mark.parametrize("variant", sorted(DEC_VARIANTS))
@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8), (20, 10), (4, 8), (10, 22)])
@pytest.mark.parametrize("L", [513, 1008, 1017, 1202, 1436])
def test_rs_reconstruct_kernel_variants_match_oracle(codec, oracle, torch, fec, tune, variant, k, m, L):
    rng = np.random.default_rng(11 * k + L + 1000 * sorted(DEC_VARIANTS).index(variant))
    n, B = k + m, 389
    S = (L + 15) // 16 * 16
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = _random_masks(rng, B, k, m)
    data_np = np.ascontiguousarray(sh[:, :k]).copy()
    for b in range(B):
        for i in range(k):
            if not (masks[b] >> i) & 1:
                data_np[b, i] = 0x3C
    par = torch.from_numpy(np.ascontiguousarray(sh[:, k:])).cuda()
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    tune(**DEC_VARIANTS[variant])
    out = torch.full((B, m, S), 0xEE, dtype=torch.uint8, device="cuda")
    data = torch.from_numpy(data_np).cuda()
    codec.rs_recover_split(k, m, data, par, dm, out, shard_len=L)
    codec.sync()
    got = out.cpu().numpy()
    for b in range(B):
        miss = [i for i in range(k) if not (masks[b] >> i) & 1]
        for r, i in enumerate(miss):
            assert np.array_equal(got[b, r, :L], sh[b, i, :L]), (b, r, i)
    codec.rs_reconstruct_split(k, m, data, par, dm, shard_len=L)
    codec.sync()
    assert np.array_equal(data.cpu().numpy()[:, :, :L], sh[:, :k, :L])


# One output slot per block (the bench's form): the direct kernel for every code whose tables it
# serves (RS(8,12), RS(4,12), RS(2,3), and RS(16,24) / RS(20,30) from the device table), mixed
# erasure counts: a block with one erased data shard is rebuilt into its slot, status 1; none
# erased, status 0; two or more with enough shards, status -1 (FEC_ERR_INVALID_ARG: more erasures
# than slots); too few shards, -4. The same semantics on the plan routes ("plan", "tile").
@pytest.mark.parametrize("variant", sorted(DEC_VARIANTS))
@pytest.mark.parametrize("k,m", [(2, 1), (8, 4), (16, 8), (20, 10), (4, 8), (10, 22)])
@pytest.mark.parametrize("L", [513, 1202])
def test_rs_recover_single_slot_variants_match_oracle(codec, oracle, torch, fec, tune, variant, k, m, L):
    rng = np.random.default_rng(3 * k + L + 100 * sorted(DEC_VARIANTS).index(variant))
    n, B = k + m, 517
    S = (L + 15) // 16 * 16
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = _random_masks(rng, B, k, m, max_loss=min(n, m + 1))
    lost = ~((masks[:, None] >> np.arange(n)[None, :]) & 1).astype(bool)
    e_d = lost[:, :k].sum(axis=1)
    few = (n - lost.sum(axis=1)) < k
    want = np.where(e_d == 0, 0, np.where(few, -4, np.where(e_d > 1, -1, 1)))
    data_np = np.ascontiguousarray(sh[:, :k]).copy()
    data_np[lost[:, :k]] = 0x3C
    data = torch.from_numpy(data_np).cuda()
    par = torch.from_numpy(np.ascontiguousarray(sh[:, k:])).cuda()
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    tune(**DEC_VARIANTS[variant])
    out = torch.full((B, 1, S), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    codec.rs_recover_split(k, m, data, par, dm, out, status=st, shard_len=L)
    if (want < 0).any():
        with pytest.raises(fec.FecError):
            codec.sync()
    else:
        codec.sync()
    assert np.array_equal(st.cpu().numpy(), want)
    got = out.cpu().numpy()
    for b in np.nonzero(want == 1)[0]:
        i = int(np.nonzero(lost[b, :k])[0][0])
        assert np.array_equal(got[b, 0, :L], sh[b, i, :L]), (b, i)


# The sorted plan kernel's two forms on codes of both sum forms: n - k < k sums over the
# complement (RS(16,24), RS(20,30) by the form compiled for the code; RS(9,10) by the general
# form), n - k >= k over the inputs (RS(4,12), RS(8,16), RS(10,32), RS(1,4)), with 1..min(k, m)
# data erasures and parity losses mixed in, over batches whose last sort window is ragged.
@pytest.mark.parametrize("k,m", [(16, 8), (20, 10), (9, 1), (4, 8), (8, 8), (10, 22), (1, 3)])
@pytest.mark.parametrize("B", [517, 9037])
def test_rs_plan_forms_match_oracle(codec, oracle, torch, tune, k, m, B):
    rng = np.random.default_rng(1000 * k + m + B)
    n, L = k + m, 1202
    S = (L + 15) // 16 * 16
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    masks = _random_masks(rng, B, k, m)
    data_np = np.ascontiguousarray(sh[:, :k]).copy()
    lost = ~((masks[:, None] >> np.arange(k)[None, :]) & 1).astype(bool)
    data_np[lost] = 0x5A
    par = torch.from_numpy(np.ascontiguousarray(sh[:, k:])).cuda()
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    tune(dec_direct=0)
    data = torch.from_numpy(data_np).cuda()
    out = torch.full((B, m, S), 0xEE, dtype=torch.uint8, device="cuda")
    codec.rs_recover_split(k, m, data, par, dm, out, shard_len=L)
    codec.sync()
    got = out.cpu().numpy()
    ne = lost.sum(axis=1)
    for b in np.flatnonzero(ne):
        miss = np.flatnonzero(lost[b])
        assert np.array_equal(got[b, :len(miss), :L], sh[b, miss, :L]), b
    codec.rs_reconstruct_split(k, m, data, par, dm, shard_len=L)
    codec.sync()
    assert np.array_equal(data.cpu().numpy()[:, :, :L], sh[:, :k, :L])


def test_rs_32_0_fully_present_is_untouched(codec, torch, fec):
    """k = 32, m = 0 (n = 32: the widest present mask): a fully present block rebuilds nothing,
    in place or out of place (klauspost ReconstructData with every shard present is a no-op)."""
    k, m, B, L, S = 32, 0, 7, 100, 112
    rng = np.random.default_rng(32)
    data_np = rng.integers(0, 256, (B, k, S), dtype=np.uint8)
    data = torch.from_numpy(data_np.copy()).cuda()
    masks = torch.from_numpy(np.full(B, 0xFFFFFFFF, dtype=np.uint32).view(np.int32)).cuda()
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    rc = codec.rs_reconstruct_raw(k, m, L, B, data.data_ptr(), k * S, data.data_ptr(), k * S, S, masks.data_ptr(),
                                  st.data_ptr(), fec.FEC_DEVICE)
    assert rc == 0
    codec.sync()
    assert np.array_equal(data.cpu().numpy(), data_np) and not st.cpu().numpy().any()
    out = torch.full((B, 1, S), 0xEE, dtype=torch.uint8, device="cuda")
    st.fill_(99)
    rc = codec.rs_recover_raw(k, m, L, B, data.data_ptr(), k * S, data.data_ptr(), k * S, S, masks.data_ptr(),
                              out.data_ptr(), S, 1, st.data_ptr())
    assert rc == 0
    codec.sync()
    assert (out.cpu().numpy() == 0xEE).all() and not st.cpu().numpy().any()
    # one erasure with no parity: too few shards, data untouched
    masks.fill_(np.uint32(0x7FFFFFFF).view(np.int32))
    rc = codec.rs_reconstruct_raw(k, m, L, B, data.data_ptr(), k * S, data.data_ptr(), k * S, S, masks.data_ptr(),
                                  st.data_ptr(), fec.FEC_DEVICE)
    assert rc == 0
    assert codec.lib_sync_rc() == fec.FEC_ERR_TOO_FEW_SHARDS
    assert (st.cpu().numpy() == fec.FEC_ERR_TOO_FEW_SHARDS).all()
    assert np.array_equal(data.cpu().numpy(), data_np)


@pytest.mark.parametrize("k,m", [(16, 8), (20, 10)])
@pytest.mark.parametrize("L", [1017, 1202])
def test_rs_recover_single_slot_big_codes(codec, oracle, torch, fec, k, m, L):
    """fec_rs_recover_batch with one output slot on RS(16,24) / RS(20,30) runs the direct kernel
    (rows by scalar loads from the device table) with no gate: blocks with one erased data shard
    are rebuilt bit-exact against the oracle, complete blocks report 0 and leave the slot alone,
    blocks with two or more erased data shards report FEC_ERR_INVALID_ARG (more erasures than
    output slots, as the plan path reports them), too-few-shards blocks FEC_ERR_TOO_FEW_SHARDS."""
    rng = np.random.default_rng(7 * k + L)
    n, B = k + m, 611
    S = (L + 15) // 16 * 16
    sh = _rand_shards(rng, B, n, S, L)
    oracle.rs_encode(k, m, sh)
    kind = rng.integers(0, 10, B)            # 0-5 single data erasure (+ parity losses), 6 none, 7-8 multi, 9 too few
    masks = np.empty(B, dtype=np.uint32)
    for b in range(B):
        lost = set()
        if kind[b] <= 5:
            lost = {int(rng.integers(0, k))} | set(int(x) for x in rng.choice(np.arange(k, n), int(kind[b] % 3), replace=False))
        elif kind[b] in (7, 8):
            lost = set(int(x) for x in rng.choice(k, int(rng.integers(2, min(k, m) + 1)), replace=False))
        elif kind[b] == 9:
            lost = set(int(x) for x in rng.choice(n, m + 1, replace=False)) | {0}
        masks[b] = ((1 << n) - 1) & ~sum(1 << i for i in lost)
    data = torch.from_numpy(np.ascontiguousarray(sh[:, :k])).cuda()
    par = torch.from_numpy(np.ascontiguousarray(sh[:, k:])).cuda()
    out = torch.full((B, 1, S), 0xEE, dtype=torch.uint8, device="cuda")
    st = torch.full((B,), 99, dtype=torch.int32, device="cuda")
    dm = torch.from_numpy(masks.view(np.int32)).cuda()
    codec.rs_recover_split(k, m, data, par, dm, out, status=st, shard_len=L)
    rc = codec.lib_sync_rc()
    got, sts = out.cpu().numpy(), st.cpu().numpy()
    for b in range(B):
        erased = [i for i in range(k) if not (masks[b] >> i) & 1]
        present = bin(int(masks[b])).count("1")
        if erased and present < k:
            assert sts[b] == fec.FEC_ERR_TOO_FEW_SHARDS, b
        elif len(erased) >= 2:
            assert sts[b] == fec.FEC_ERR_INVALID_ARG, b
        elif len(erased) == 1:
            assert sts[b] == 1 and np.array_equal(got[b, 0, :L], sh[b, erased[0], :L]), b
        else:
            assert sts[b] == 0 and (got[b] == 0xEE).all(), b
    assert rc != 0   # the batch held failing blocks: the sticky error says so


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("chunk", [0, 7])
@pytest.mark.parametrize("k,m,L", [(2, 1, 1202), (8, 4, 1202), (16, 8, 700), (20, 10, 1436), (8, 4, 33)])
def test_rs_host_pipeline_matches_oracle(codec, oracle, torch, fec, pinned, chunk, k, m, L):
    """FEC_HOST (pageable, staged) and FEC_HOST_PINNED (direct 2D DMA) through the two-set
    pipeline, with many small chunks (chunk = 7 blocks) so consecutive chunks alternate sets and
    overlap: encode, then in-place reconstruct of random erasures (some blocks unrecoverable, some
    complete) with split data / parity buffers of a padded host layout, against the oracle."""
    rng = np.random.default_rng(k * 100 + L + chunk + pinned)
    n, B, S = k + m, 97, L + 5                           # unaligned host stride: any layout
    full = np.zeros((B, n, L), dtype=np.uint8)
    full[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    oracle.rs_encode(k, m, full)
    mk = (lambda a: torch.from_numpy(a).pin_memory()) if pinned else (lambda a: a)
    get = (lambda t: t.numpy()) if pinned else (lambda a: a)
    data = np.zeros((B, k, S), dtype=np.uint8)
    data[:, :, :L] = full[:, :k]
    data = mk(data)
    par = mk(np.full((B, m, S), 0x77, dtype=np.uint8))
    old = codec.set_tuning(host_chunk=chunk)
    try:
        codec.rs_encode_split(k, m, data, par, shard_len=L)
        assert np.array_equal(get(par)[:, :, :L], full[:, k:])
        assert (get(par)[:, :, L:] == 0x77).all()        # exactly shard_len bytes written
        masks = _random_masks(rng, B, k, m, max_loss=m + 1)
        dmg = get(data).copy()
        for b in range(B):
            for i in range(k):
                if not (masks[b] >> i) & 1:
                    dmg[b, i, :L] = 0xA1
        want = np.zeros((B, n, L), dtype=np.uint8)
        want[:, :k] = dmg[:, :, :L]
        want[:, k:] = full[:, k:]
        st_want = oracle.rs_reconstruct(k, m, want, masks)
        d2 = mk(dmg)
        st = np.full(B, 7, dtype=np.int32)
        rc = codec.rs_reconstruct_split(k, m, d2, par, masks, status=st, shard_len=L)
        assert rc == (fec.FEC_ERR_TOO_FEW_SHARDS if (st_want != 0).any() else fec.FEC_OK)
        assert np.array_equal(st != 0, st_want != 0)
        assert np.array_equal(get(d2)[:, :, :L], want[:, :k])
        assert (get(d2)[:, :, L:] == dmg[:, :, L:]).all()
    finally:
        codec.set_tuning(**old)


@pytest.mark.parametrize("pinned", [False, True])
def test_xor_host_pipeline_matches_oracle(codec, oracle, torch, fec, pinned):
    rng = np.random.default_rng(5 + pinned)
    k, B, L = 3, 61, 1202
    sh = np.zeros((B, k + 1, L), dtype=np.uint8)
    sh[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    ref = oracle.xor_encode(k, sh.copy())
    buf = torch.from_numpy(sh.copy()).pin_memory() if pinned else sh.copy()
    old = codec.set_tuning(host_chunk=5)
    try:
        codec.xor_encode(k, buf)
    finally:
        codec.set_tuning(**old)
    got = buf.numpy() if pinned else buf
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("k,m,chunk", [(8, 4, 61), (16, 8, 37), (20, 10, 64)])
def test_rs_host_pipeline_many_chunks_multi_erasure(codec, oracle, fec, k, m, chunk):
    """Host-path reconstruct over many small chunks (consecutive chunks run on the two staging
    sets' streams at once) with up to m erasures per block: the plan records are per stream, so
    overlapping chunks never share one. Checked against the oracle block by block."""
    rng = np.random.default_rng(7000 + k + chunk)
    n, B, L = k + m, 1500, 600
    full = np.zeros((B, n, L), dtype=np.uint8)
    full[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    oracle.rs_encode(k, m, full)
    masks = _random_masks(rng, B, k, m, max_loss=m)
    dmg = full[:, :k].copy()
    for b in range(B):
        for i in range(k):
            if not (masks[b] >> i) & 1:
                dmg[b, i] = 0xA1
    par = full[:, k:].copy()
    old = codec.set_tuning(host_chunk=chunk)
    try:
        st = np.full(B, 7, dtype=np.int32)
        rc = codec.rs_reconstruct_split(k, m, dmg, par, masks, status=st, shard_len=L)
        assert rc == fec.FEC_OK and (st == 0).all()
        assert np.array_equal(dmg, full[:, :k])
    finally:
        codec.set_tuning(**old)


@pytest.mark.parametrize("threads,chunk", [(8, 0), (3, 1100), (16, 600), (5, 0)])
def test_rs_host_copy_pool_matches_oracle(codec, oracle, fec, threads, chunk):
    """FEC_HOST (pageable) with chunks of >= 512 blocks, whose staging and scatter copies run on
    the persistent copy workers, with 3..16 parts and one chunk or several. Encode and a
    multi-erasure reconstruct against the oracle."""
    rng = np.random.default_rng(300 + threads + chunk)
    k, m, B, L = 8, 4, 3000, 600
    n = k + m
    full = np.zeros((B, n, L), dtype=np.uint8)
    full[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    oracle.rs_encode(k, m, full)
    old = codec.set_tuning(host_threads=threads, host_chunk=chunk)
    try:
        data = full[:, :k].copy()
        par = np.zeros((B, m, L), dtype=np.uint8)
        codec.rs_encode_split(k, m, data, par, shard_len=L)
        assert np.array_equal(par, full[:, k:])
        masks = _random_masks(rng, B, k, m, max_loss=m)
        dmg = full[:, :k].copy()
        lost = ~((masks[:, None] >> np.arange(k)[None, :]) & 1).astype(bool)
        dmg[lost] = 0xA1
        st = np.full(B, 7, dtype=np.int32)
        rc = codec.rs_reconstruct_split(k, m, dmg, par, masks, status=st, shard_len=L)
        assert rc == fec.FEC_OK and (st == 0).all()
        assert np.array_equal(dmg, full[:, :k])
    finally:
        codec.set_tuning(**old)


def test_host_staging_release_and_regrow(codec, oracle, fec):
    """fec_ctx_release_staging frees the host path's staging sets between calls; calls before and
    after it (a mid-sized call split over the three sets, then a small one) stay exact."""
    rng = np.random.default_rng(77)
    k, m, L = 8, 4, 1202
    for B in (20000, 300, 7000):
        full = np.zeros((B, k + m, L), dtype=np.uint8)
        full[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
        oracle.rs_encode(k, m, full)
        data = full[:, :k].copy()
        par = np.zeros((B, m, L), dtype=np.uint8)
        codec.rs_encode_split(k, m, data, par, shard_len=L)
        assert np.array_equal(par, full[:, k:])
        masks = _random_masks(rng, B, k, m, max_loss=m)
        dmg = full[:, :k].copy()
        dmg[~((masks[:, None] >> np.arange(k)[None, :]) & 1).astype(bool)] = 0xA1
        st = np.full(B, 7, dtype=np.int32)
        assert codec.rs_reconstruct_split(k, m, dmg, par, masks, status=st, shard_len=L) == fec.FEC_OK
        assert (st == 0).all() and np.array_equal(dmg, full[:, :k])
        codec.release_staging()
        codec.release_staging()   # twice: a no-op


def test_rs_host_copy_pool_concurrent_contexts(oracle, fec):
    """Two contexts on two threads in FEC_HOST calls at once: one gets the persistent copy
    workers, the other finds them busy and copies on threads of its own; both results exact."""
    import threading
    k, m, B, L = 8, 4, 2000, 900
    rng = np.random.default_rng(99)
    full = np.zeros((B, k + m, L), dtype=np.uint8)
    full[:, :k] = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    oracle.rs_encode(k, m, full)
    errs = []

    def worker(seed):
        c = fec.Codec(0)
        try:
            for _ in range(6):
                data = full[:, :k].copy()
                par = np.zeros((B, m, L), dtype=np.uint8)
                c.rs_encode_split(k, m, data, par, shard_len=L)
                if not np.array_equal(par, full[:, k:]):
                    errs.append("encode %d" % seed)
        except Exception as e:   # reported below, in the main thread
            errs.append(repr(e))
        finally:
            c.close()

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts)
    assert not errs, errs


def test_stream_switch_orders_shared_workspace(fec, torch):
    """fec_ctx_set_stream between two launches that share the ctx's workspace (the RS(16,24)
    plan records): the second stream must not rewrite the records while the first stream's
    rebuild still reads them. Two multi-erasure batches, one per torch stream, launched back to
    back; both must come back equal to the original data (round trip; the kernels themselves
    are checked against the oracle above)."""
    k, m, L, S = 16, 8, 1202, 1216
    n = k + m
    c = fec.Codec(0)
    try:
        outs = []
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for i, B in enumerate((1 << 16, 1 << 15)):
            rng = np.random.default_rng(0x57 + i)
            sh = torch.zeros((B, n, S), dtype=torch.uint8, device="cuda")
            sh[:, :k, :L] = torch.from_numpy(rng.integers(0, 256, (B, k, L), dtype=np.uint8)).cuda()
            # the data was written on torch's stream; the codec's streams are non-blocking and do
            # not order after it (the first batch was only saved by the table upload's device sync)
            torch.cuda.synchronize()
            c.set_stream(streams[i].cuda_stream)
            c.rs_encode(k, m, sh, shard_len=L)
            c.sync()
            masks = _random_masks(rng, B, k, m, max_loss=m)
            lost = torch.from_numpy(((masks[:, None] >> np.arange(n)) & 1) == 0).cuda()
            outs.append((sh.clone(), sh, lost, torch.from_numpy(masks.view(np.int32)).cuda()))
        for i, (want, sh, lost, dm) in enumerate(outs):
            sh[lost] = 0x5A
        torch.cuda.synchronize()
        for i, (want, sh, lost, dm) in enumerate(outs):   # back to back, no host wait between
            c.set_stream(streams[i].cuda_stream)
            c.rs_reconstruct(k, m, sh, dm, shard_len=L)
        torch.cuda.synchronize()
        assert c.lib_sync_rc() == 0
        for want, sh, lost, dm in outs:
            assert torch.equal(sh[:, :k, :L], want[:, :k, :L])
    finally:
        c.close()
