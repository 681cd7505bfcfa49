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


@pytest.mark.parametrize("zc", [0, 1 << 30])   # knob bat_zc: the copy form, every set zero-copy
@pytest.mark.parametrize("scheme,k,m", [(RS, 8, 4), (RS, 20, 10), (RS, 2, 1), (XOR, 4, 1)])
def test_submit_ref_matches_oracle(fec, oracle, tune, scheme, k, m, zc):
    tune(bat_zc=zc)
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


def _bind_dec(lib):
    _bind(lib)
    lib.fec_go_decoder_new.restype = _vp
    lib.fec_go_decoder_new.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _sz, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_int)]
    lib.fec_go_decoder_free.argtypes = [_vp]
    lib.fec_go_decoder_free.restype = None
    for fn in (lib.fec_go_decoder_submit, lib.fec_go_decoder_submit_ref):
        fn.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(_vp),
                       ctypes.POINTER(_sz), ctypes.POINTER(_vp), ctypes.POINTER(_sz), ctypes.POINTER(ctypes.c_int)]
    lib.fec_go_decoder_poll.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                        ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                        _sz, _sz, ctypes.POINTER(_sz)]
    return lib


@pytest.mark.parametrize("zc", [0, 1 << 30])   # knob bat_zc: the copy form, every set zero-copy
@pytest.mark.parametrize("k,m", [(8, 4), (20, 10), (2, 1)])
def test_decoder_submit_ref_matches_oracle(fec, oracle, tune, k, m, zc):
    """fec_go_decoder_submit_ref: received sources and repairs in registered packet buffers are
    gathered by the device (sources framed with their trailer at `biggest`, repairs verbatim).
    Every polled payload must equal the oracle's recoverSymbolPayloads (reed_solomon.go:92-136)
    for the same block, with referenced, copied (outside the pool) and empty (missing) shards
    mixed, at unaligned offsets, over several batches of both staging sets."""
    tune(bat_zc=zc)
    lib = _bind_dec(fec.lib)
    rng = np.random.default_rng(0xDEC + 31 * k + m)
    nblocks, maxb, n = 200, 32, k + m
    nbuf = nblocks * n + 8
    base = _vp()
    err = ctypes.c_int(0)
    pool = lib.fec_go_pool_new(nbuf, ctypes.byref(base), ctypes.byref(err))
    assert pool, lib.fec_last_error()
    dec = lib.fec_go_decoder_new(RS, k, m, maxb, 0, ctypes.byref(err))
    assert dec, lib.fec_last_error()
    outside = []
    try:
        pool_np = np.frombuffer((ctypes.c_uint8 * (nbuf * POOL_SLOT)).from_address(base.value), dtype=np.uint8)
        ptrs = (_vp * n)()
        lens = (_sz * n)()
        staged = ctypes.c_int(0)
        ids = (ctypes.c_uint64 * maxb)()
        pl = (ctypes.c_uint32 * maxb)()
        offs = (ctypes.c_uint64 * maxb)()
        out = np.zeros(maxb * k * SLOT, dtype=np.uint8)
        nb = _sz(0)
        want, got, order = {}, {}, []

        def poll(wait):
            assert lib.fec_go_decoder_poll(dec, wait, ids, pl, offs, out.ctypes.data, out.size, maxb,
                                           ctypes.byref(nb)) == 0, lib.fec_last_error()
            for d in range(nb.value):
                order.append(ids[d])
                got[ids[d]] = bytes(out[offs[d]:offs[d] + pl[d]])

        def place(slot, data, mode, i):
            if mode == 3 and i % 2:   # outside any pool: copied by the library
                arr = np.frombuffer(bytearray(data) + b"\0" * 16, dtype=np.uint8).copy()
                outside.append(arr)
                return arr.ctypes.data
            off = 2 * int(rng.integers(1, 4)) if mode == 2 else 0
            start = slot * POOL_SLOT + off
            if len(data) + off > POOL_SLOT:
                start -= off
            pool_np[start:start + len(data)] = np.frombuffer(data, dtype=np.uint8)
            return base.value + start

        for b in range(nblocks):
            mode = b % 5    # 0,1: all in the pool; 2: unaligned; 3: mixed with copied; 4: an empty repair
            pls = [rng.integers(0, 256, int(rng.integers(1, 1201)), dtype=np.uint8).tobytes() for _ in range(k)]
            reps = _oracle_repairs(oracle, RS, k, m, pls)
            L = len(reps[0])
            lost = set(rng.choice(k, size=int(rng.integers(1, m + 1)), replace=False).tolist())
            keep = sorted(rng.choice(m, size=m, replace=False).tolist()[:max(len(lost), 1) + int(rng.integers(0, 2))])
            empty = keep[0] if mode == 4 and len(keep) > len(lost) else None
            src = {}
            for i in range(k):
                if i in lost:
                    ptrs[i], lens[i] = None, 0
                else:
                    ptrs[i], lens[i] = place(b * n + i, pls[i], mode, i), len(pls[i])
                    src[b * k + i] = oracle.Payload(pls[i], 1452)
            rmap = {}
            for p in range(m):
                if p not in keep:
                    ptrs[k + p], lens[k + p] = None, 0
                elif p == empty:
                    ptrs[k + p], lens[k + p] = base.value + (b * n + k + p) * POOL_SLOT, 0
                    rmap[p] = oracle.Payload(b"", 0)
                else:
                    ptrs[k + p], lens[k + p] = place(b * n + k + p, reps[p], mode, p), L
                    rmap[p] = oracle.Payload(reps[p], L)
            ob = oracle.Block(id=b, tot_src=k, tot_rep=m, biggest=L - 2, smallest=b * k, largest=b * k + k - 1,
                              sources=src, repairs=rmap)
            exp, e = oracle.rs_recover_symbol_payloads(ob, k, m)
            rsrc = ctypes.cast(ptrs, ctypes.POINTER(_vp))
            rrep = ctypes.cast(ctypes.byref(ptrs, k * ctypes.sizeof(_vp)), ctypes.POINTER(_vp))
            rlen = ctypes.cast(ctypes.byref(lens, k * ctypes.sizeof(_sz)), ctypes.POINTER(_sz))
            rc = lib.fec_go_decoder_submit_ref(dec, b, b * k, b * k + k - 1, L - 2, rsrc, lens, rrep, rlen,
                                               ctypes.byref(staged))
            if e is not None:
                assert rc != 0, (b, e)
                continue
            assert rc == 0, lib.fec_last_error()
            assert staged.value == 1
            want[b] = exp
            if b % 29 == 28:
                poll(0)
        while len(got) < len(want):
            before = len(got)
            poll(1)
            assert len(got) > before
        assert order == sorted(want), "blocks come back in submission order"
        for b, exp in want.items():
            assert got[b] == exp, "block %d" % b
    finally:
        lib.fec_go_decoder_free(dec)
        lib.fec_go_pool_free(pool)
