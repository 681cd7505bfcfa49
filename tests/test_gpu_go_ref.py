"""The Go ABI's by-reference encoder path (include/fec_go.h fec_go_pool_new /
fec_go_encoder_submit_ref): payloads in registered packet buffers are gathered and framed by
the device (fec_pack.hip gather_desc_kernel) instead of copied by the host. Every polled repair
payload must equal the CPU oracle's repairSymbols (reed_solomon.go:26-68, xor.go:14-56) for the
same block, whether its payloads were referenced, copied (outside any pool) or a mix, at
unaligned buffer offsets, zero lengths and batches that split across staging sets."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SLOT = 1452          # FEC_GO_SLOT
POOL_SLOT = 1456     # FEC_GO_POOL_SLOT
RS, XOR = 2, 1       # FEC_SCHEME_REED_SOLOMON, FEC_SCHEME_XOR

_vp, _sz = ctypes.c_void_p, ctypes.c_size_t


def _bind(lib):
    lib.fec_go_pool_new.restype = _vp
    lib.fec_go_pool_new.argtypes = [_sz, ctypes.POINTER(_vp), ctypes.POINTER(ctypes.c_int)]
    lib.fec_go_pool_free.argtypes = [_vp]
    lib.fec_go_pool_free.restype = None
    lib.fec_go_encoder_new.restype = _vp
    lib.fec_go_encoder_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _sz, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int)]
    lib.fec_go_encoder_free.argtypes = [_vp]
    lib.fec_go_encoder_free.restype = None
    for fn in (lib.fec_go_encoder_submit, lib.fec_go_encoder_submit_ref):
        fn.argtypes = [_vp, ctypes.c_uint64, ctypes.POINTER(_vp), ctypes.POINTER(_sz), ctypes.c_int]
    lib.fec_go_encoder_poll.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.c_void_p, _sz, ctypes.POINTER(_sz)]
    lib.fec_last_error.restype = ctypes.c_char_p
    return lib


def _oracle_repairs(oracle, scheme, k, m, payloads):
    b = oracle.Block(id=0, tot_src=k, tot_rep=m, biggest=max(len(p) for p in payloads), smallest=0,
                     largest=k - 1, sources={i: oracle.Payload(p, 1452) for i, p in enumerate(payloads)})
    frames, err = (oracle.rs_repair_symbols(b, k, m) if scheme == RS else oracle.xor_repair_symbols(b))
    assert err is None, err
    return [f[2] for f in frames]


@pytest.mark.parametrize("scheme,k,m", [(RS, 8, 4), (RS, 20, 10), (RS, 2, 1), (XOR, 4, 1)])
def test_submit_ref_matches_oracle(fec, oracle, scheme, k, m):
    lib = _bind(fec.lib)
    rng = np.random.default_rng(0x9A7 + 31 * k + m)
    nblocks, maxb = 300, 64          # several batches of both staging sets
    nbuf = nblocks * k + 8
    base = _vp()
    err = ctypes.c_int(0)
    pool = lib.fec_go_pool_new(nbuf, ctypes.byref(base), ctypes.byref(err))
    assert pool, lib.fec_last_error()
    enc = lib.fec_go_encoder_new(scheme, k, m, maxb, 0, ctypes.byref(err))
    assert enc, lib.fec_last_error()
    outside = []     # payload buffers outside the pool (copied by the library)
    try:
        pool_mem = (ctypes.c_uint8 * (nbuf * POOL_SLOT)).from_address(base.value)
        pool_np = np.frombuffer(pool_mem, dtype=np.uint8)
        want = {}
        ptrs = (_vp * k)()
        lens = (_sz * k)()
        got_ids, got = [], {}
        ids = (ctypes.c_uint64 * maxb)()
        rl = (ctypes.c_uint32 * maxb)()
        rep = np.zeros(maxb * m * SLOT, dtype=np.uint8)
        n = _sz(0)

        def poll(wait):
            assert lib.fec_go_encoder_poll(enc, wait, ids, rl, rep.ctypes.data, maxb, ctypes.byref(n)) == 0, \
                lib.fec_last_error()
            for d in range(n.value):
                got_ids.append(ids[d])
                got[ids[d]] = [bytes(rep[(d * m + i) * SLOT:(d * m + i) * SLOT + rl[d]]) for i in range(m)]

        for b in range(nblocks):
            mode = b % 5    # 0,1: all in the pool; 2: unaligned offsets; 3: mixed with copied; 4: short/zero
            biggest_cap = 1200 if mode != 4 else 40
            pls = []
            for i in range(k):
                ln = int(rng.integers(0, biggest_cap + 1)) if mode >= 3 or i == 0 else biggest_cap
                pls.append(rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
            for i, p in enumerate(pls):
                slot = b * k + i
                off = 2 * int(rng.integers(1, 4)) if mode == 2 else 0   # 2-byte aligned, as sliced payloads
                if mode == 3 and i % 2:
                    arr = np.frombuffer(bytearray(p) + b"\0" * 16, dtype=np.uint8).copy()
                    outside.append(arr)
                    ptrs[i] = arr.ctypes.data
                else:
                    start = slot * POOL_SLOT + off
                    if len(p) + off > POOL_SLOT:
                        start -= off
                    pool_np[start:start + len(p)] = np.frombuffer(p, dtype=np.uint8)
                    ptrs[i] = base.value + start
                lens[i] = len(p)
            want[b] = _oracle_repairs(oracle, scheme, k, m, pls)
            rc = lib.fec_go_encoder_submit_ref(enc, b, ptrs, lens, k)
            assert rc == 0, lib.fec_last_error()
            if b % 37 == 36:
                poll(0)
        while len(got) < nblocks:
            before = len(got)
            poll(1)
            assert len(got) > before
        assert got_ids == list(range(nblocks)), "blocks come back in submission order"
        for b in range(nblocks):
            assert got[b] == want[b], "block %d" % b
    finally:
        lib.fec_go_encoder_free(enc)
        lib.fec_go_pool_free(pool)


def test_submit_ref_errors_match_submit(fec):
    """The reference's repairSymbols checks, in order, for the by-reference form: an incomplete
    block and an oversized payload fail exactly as fec_go_encoder_submit does."""
    lib = _bind(fec.lib)
    err = ctypes.c_int(0)
    base = _vp()
    pool = lib.fec_go_pool_new(16, ctypes.byref(base), ctypes.byref(err))
    enc = lib.fec_go_encoder_new(RS, 4, 2, 8, 0, ctypes.byref(err))
    try:
        ptrs = (_vp * 4)(*[base.value + i * POOL_SLOT for i in range(4)])
        for count, lens in ((3, [10, 10, 10, 10]), (4, [10, 1500, 10, 10])):
            ln = (_sz * 4)(*lens)
            r1 = lib.fec_go_encoder_submit(enc, 1, ptrs, ln, count)
            e1 = lib.fec_last_error()
            r2 = lib.fec_go_encoder_submit_ref(enc, 1, ptrs, ln, count)
            e2 = lib.fec_last_error()
            assert r1 != 0 and (r1, e1) == (r2, e2)
    finally:
        lib.fec_go_encoder_free(enc)
        lib.fec_go_pool_free(pool)
