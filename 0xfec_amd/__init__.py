"""0xfec_amd — MI355X-native block FEC engine (the hot path of ddritzenhoff/0xFEC internal/fec).

The compute lives in lib0xfec_hip.so (hand-written gfx950 HIP kernels behind the C ABI of
include/fec_hip.h). This module is a thin ctypes face of that ABI, plus the host-side mirror
of the reference's scheme/manager layer (see `scheme`). There is no CPU fallback: if the
library is missing the import fails, and without a HIP device every compute call raises.

Import by name (the directory starts with a digit):
    fec = importlib.import_module("0xfec_amd")
"""
import ctypes
import os

# PyTorch-ROCm ships its own libamdhip64.so (same SONAME, libamdhip64.so.7). Loading torch
# first makes the dynamic linker bind this library to that one runtime, so device pointers,
# streams and events are shared with torch; loading ours first would start a second HIP
# runtime in the process, and torch then finds no GPU. Without torch (e.g. a cgo host) the
# library binds to /opt/rocm's runtime.
try:
    import torch as _torch  # noqa: F401
except ImportError:
    _torch = None

from ._build import LIB as _LIB_PATH

# FEC_LIB_PATH selects another build of the same library: the host-ASan/UBSan build
# (0xfec_amd/_san/lib0xfec_hip_san.so) that tests/test_sanitizers.py runs the CPU suite against
_LIB_PATH = os.environ.get("FEC_LIB_PATH") or _LIB_PATH

if not os.path.exists(_LIB_PATH):
    raise ImportError("lib0xfec_hip.so not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                      "(or python 0xfec_amd/_build.py)")

lib = ctypes.CDLL(_LIB_PATH)

# --- return codes / flags (include/fec_hip.h)
FEC_OK = 0
FEC_ERR_INVALID_ARG = -1
FEC_ERR_INV_SHARD_NUM = -2
FEC_ERR_MAX_SHARD_NUM = -3
FEC_ERR_TOO_FEW_SHARDS = -4
FEC_ERR_SHARD_SIZE = -5
FEC_ERR_SHARD_NO_DATA = -6
FEC_ERR_ALIGNMENT = -7
FEC_ERR_HIP = -8
FEC_ERR_NOMEM = -9
FEC_ERR_NO_DEVICE = -10
FEC_DEVICE = 0
FEC_HOST = 1
FEC_HOST_PINNED = 2
FEC_MAX_DECODE_SHARDS = 32

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i = ctypes.c_int

lib.fec_version.restype = ctypes.c_char_p
lib.fec_strerror.restype = ctypes.c_char_p
lib.fec_strerror.argtypes = [_i]
lib.fec_device_count.argtypes = [ctypes.POINTER(_i)]
lib.fec_ctx_create.argtypes = [_i, ctypes.POINTER(_vp)]
lib.fec_ctx_destroy.argtypes = [_vp]
lib.fec_ctx_destroy.restype = None
lib.fec_ctx_set_stream.argtypes = [_vp, _vp]
lib.fec_ctx_reset_stream.argtypes = [_vp]
lib.fec_ctx_release_staging.argtypes = [_vp]
lib.fec_ctx_stream.argtypes = [_vp]
lib.fec_ctx_stream.restype = _vp
lib.fec_sync.argtypes = [_vp]
lib.fec_rs_matrix.argtypes = [_i, _i, _vp]
lib.fec_rs_prepare.argtypes = [_vp, _i, _i]
lib.fec_rs_encode_batch.argtypes = [_vp, _i, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _i]
lib.fec_rs_reconstruct_batch.argtypes = [_vp, _i, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _vp, _vp, _i]
lib.fec_rs_recover_batch.argtypes = [_vp, _i, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _vp, _vp, _sz, _i, _vp, _i]
lib.fec_xor_encode_batch.argtypes = [_vp, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _i]
lib.fec_xor_reconstruct_batch.argtypes = [_vp, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _vp, _vp, _i]
_u64 = ctypes.c_uint64
lib.fec_synth_data.argtypes = [_vp, _u64, _u64, _sz, _i, _sz, _vp, _sz, _sz]
lib.fec_synth_single_erasures.argtypes = [_vp, _u64, _u64, _sz, _i, _i, _vp, _vp]
lib.fec_probe_encode_traffic.argtypes = [_vp, _i, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _i]
lib.fec_probe_recover_traffic.argtypes = [_vp, _i, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _vp, _vp, _sz, _i]
lib.fec_probe_rebuild_traffic.argtypes = [_vp, _i, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _vp, _vp, _sz, _i]
lib.fec_probe_stream_traffic.argtypes = [_vp, _i, _sz, _sz, _vp, _sz, _vp, _sz, _sz, _i]
lib.fec_probe_link.argtypes = [_vp, _sz, _i, ctypes.POINTER(ctypes.c_double)]


class FecError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = lib.fec_strerror(code).decode()
        super().__init__("%s%s (code %d)" % (what + ": " if what else "", msg, code))


def _check(rc, what=""):
    if rc != FEC_OK:
        raise FecError(rc, what)
    return rc


def version():
    return lib.fec_version().decode()


def device_count():
    n = _i(0)
    lib.fec_device_count(ctypes.byref(n))
    return n.value


def rs_matrix(k, m):
    """n x k systematic matrix of RS(k, m) (klauspost reedsolomon.New default); no device."""
    import numpy as np
    out = np.zeros((k + m, k), dtype=np.uint8)
    _check(lib.fec_rs_matrix(k, m, out.ctypes.data), "fec_rs_matrix")
    return out


def _addr(x):
    """(address, memory kind) for a numpy array, a torch tensor, or a raw device address."""
    if isinstance(x, int):
        return x, FEC_DEVICE
    mod = type(x).__module__
    if mod.startswith("numpy"):
        return x.ctypes.data, FEC_HOST
    if mod.startswith("torch"):
        if x.is_cuda:
            return x.data_ptr(), FEC_DEVICE
        return x.data_ptr(), (FEC_HOST_PINNED if x.is_pinned() else FEC_HOST)
    raise TypeError("unsupported buffer type %r" % type(x))


def _shape3(shards):
    B, n, S = shards.shape
    if hasattr(shards, "is_contiguous"):
        assert shards.is_contiguous()
    else:
        assert shards.flags.c_contiguous
    return B, n, S


class Codec:
    """One device context (one HIP stream). Batch entry points over [B, n, S] uint8 arrays:
    numpy arrays and pageable CPU tensors run the FEC_HOST path (staged through pinned memory),
    pinned CPU tensors the FEC_HOST_PINNED path (direct DMA), CUDA tensors the FEC_DEVICE path
    (asynchronous on the ctx stream; call sync())."""

    def __init__(self, device=0):
        h = _vp()
        _check(lib.fec_ctx_create(device, ctypes.byref(h)), "fec_ctx_create")
        self._h = h
        self.device = device

    def close(self):
        if self._h:
            lib.fec_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def stream(self):
        return lib.fec_ctx_stream(self._h)

    def set_stream(self, stream_ptr):
        """Enqueue on an external hipStream_t (0/None = the null stream)."""
        _check(lib.fec_ctx_set_stream(self._h, stream_ptr or None))

    def reset_stream(self):
        _check(lib.fec_ctx_reset_stream(self._h))

    def use_torch_stream(self):
        """Enqueue on torch's current stream of this device, so codec calls order naturally
        with torch ops on the same tensors."""
        import torch
        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)
        return self

    def sync(self):
        return _check(lib.fec_sync(self._h), "fec_sync")

    def release_staging(self):
        """Free the host-path staging sets (fec_ctx_release_staging); the next host call makes them."""
        return _check(lib.fec_ctx_release_staging(self._h), "fec_ctx_release_staging")

    def lib_sync_rc(self):
        """fec_sync's return code (FEC_ERR_TOO_FEW_SHARDS after a failed block) without raising."""
        return lib.fec_sync(self._h)

    # Tuning knobs (tests and tools; defaults are the measured best): residency of the shipped
    # kernels, routing among shipped kernels, host-path sizes. Keys of the library's internal,
    # test-only fec__set_tuning() in fk::Tuning's declaration order (fec_kernels.hpp); the setting
    # is process-wide.
    TUNING_KEYS = {"enc_wpc": 0, "gen_wpc": 1, "dec_wpc": 2, "dir_wpc": 3, "enc_bwpc": 4, "enc_fixed": 5,
                   "dec_wave": 6, "dec_direct": 7, "host_chunk": 8, "host_threads": 9, "bat_zc": 10,
                   "dec_route": 11, "st_pol": 12, "dst_pol": 13,
                   "route_wpc": 14, "route_ww": 15, "xor_wpc": 16, "enc_ww": 17}

    def set_tuning(self, **knobs):
        """Set kernel-selection knobs; returns the previous values (pass them back to restore)."""
        fn = lib.fec__set_tuning
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        fn.restype = ctypes.c_int
        old = {}
        for name, val in knobs.items():
            old[name] = fn(self._h, self.TUNING_KEYS[name], int(val))
        return old

    def prepare(self, k, m):
        return _check(lib.fec_rs_prepare(self._h, k, m), "fec_rs_prepare")

    # ---- raw C-ABI mirrors (addresses + strides)
    def rs_encode_raw(self, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, flags):
        return _check(lib.fec_rs_encode_batch(self._h, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, flags),
                      "fec_rs_encode_batch")

    def rs_reconstruct_raw(self, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, masks, status, flags):
        return lib.fec_rs_reconstruct_batch(self._h, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss,
                                            masks, status, flags)

    # ---- array conveniences. Interleaved form: shards is [B, k+m, S]. Split form: data
    # [B, k, S] and parity [B, m, S] in separate buffers. shard_len defaults to S.
    def rs_encode(self, k, m, shards, shard_len=None):
        B, n, S = _shape3(shards)
        assert n == k + m
        a, kind = _addr(shards)
        L = S if shard_len is None else shard_len
        return self.rs_encode_raw(k, m, L, B, a, n * S, a + k * S, n * S, S, kind)

    def rs_encode_split(self, k, m, data, parity, shard_len=None):
        B, kk, S = _shape3(data)
        B2, mm, S2 = _shape3(parity)
        assert (kk, mm, B, S) == (k, m, B2, S2)
        d, kind = _addr(data)
        p, kind2 = _addr(parity)
        assert kind == kind2
        L = S if shard_len is None else shard_len
        return self.rs_encode_raw(k, m, L, B, d, k * S, p, m * S, S, kind)

    def _recon(self, fn, what, k, m, B, S, d, dbs, p, pbs, kind, masks, status, shard_len):
        ma, mkind = _addr(masks)
        assert (mkind == FEC_DEVICE) == (kind == FEC_DEVICE), "masks must live where the shards live"
        sa = _addr(status)[0] if status is not None else None
        L = S if shard_len is None else shard_len
        rc = fn(B, L, d, dbs, p, pbs, S, ma, sa, kind)
        if rc not in (FEC_OK, FEC_ERR_TOO_FEW_SHARDS):
            _check(rc, what)
        return rc

    def rs_reconstruct(self, k, m, shards, masks, status=None, shard_len=None):
        """Returns the C return code (FEC_OK or FEC_ERR_TOO_FEW_SHARDS for FEC_HOST)."""
        B, n, S = _shape3(shards)
        assert n == k + m
        a, kind = _addr(shards)
        fn = lambda B_, L, d, dbs, p, pbs, ss, ma, sa, kd: lib.fec_rs_reconstruct_batch(
            self._h, k, m, L, B_, d, dbs, p, pbs, ss, ma, sa, kd)
        return self._recon(fn, "fec_rs_reconstruct_batch", k, m, B, S, a, n * S, a + k * S, n * S, kind,
                           masks, status, shard_len)

    def rs_reconstruct_split(self, k, m, data, parity, masks, status=None, shard_len=None):
        B, kk, S = _shape3(data)
        assert kk == k and tuple(parity.shape) == (B, m, S)
        d, kind = _addr(data)
        p, _ = _addr(parity)
        fn = lambda B_, L, d_, dbs, p_, pbs, ss, ma, sa, kd: lib.fec_rs_reconstruct_batch(
            self._h, k, m, L, B_, d_, dbs, p_, pbs, ss, ma, sa, kd)
        return self._recon(fn, "fec_rs_reconstruct_batch", k, m, B, S, d, k * S, p, m * S, kind,
                           masks, status, shard_len)

    def rs_recover_raw(self, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, masks, out, out_bs, out_slots,
                       status, flags=FEC_DEVICE):
        return lib.fec_rs_recover_batch(self._h, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, masks,
                                        out, out_bs, out_slots, status, flags)

    def rs_recover_split(self, k, m, data, parity, masks, out, status=None, shard_len=None):
        """Rebuild the erased data shards of each block into out [B, slots, S] (ascending order);
        status[b] = number rebuilt, or a negative error code."""
        B, kk, S = _shape3(data)
        B2, slots, S2 = _shape3(out)
        assert kk == k and tuple(parity.shape) == (B, m, S) and (B2, S2) == (B, S)
        L = S if shard_len is None else shard_len
        sa = _addr(status)[0] if status is not None else None
        rc = self.rs_recover_raw(k, m, L, B, _addr(data)[0], k * S, _addr(parity)[0], m * S, S, _addr(masks)[0],
                                 _addr(out)[0], slots * S, slots, sa)
        return _check(rc, "fec_rs_recover_batch")

    # ---- synthetic workload on the device (include/fec_synth.h; same bytes as shard.py)
    def synth_data(self, seed, first_block, nblocks, k, payload_len, data, block_stride, shard_stride):
        """Fill data shards of global blocks [first_block, first_block + nblocks) at the device
        address `data` (asynchronous on the ctx stream)."""
        return _check(lib.fec_synth_data(self._h, seed, first_block, nblocks, k, payload_len, data, block_stride,
                                         shard_stride), "fec_synth_data")

    def synth_single_erasures(self, seed, first_block, nblocks, k, m, masks, erased=None):
        return _check(lib.fec_synth_single_erasures(self._h, seed, first_block, nblocks, k, m, masks, erased),
                      "fec_synth_single_erasures")

    # ---- traffic twins of the headline kernels (include/fec_probe.h; measurement only). wpc:
    # resident workgroups per CU (-1: the twinned kernel's own, 0: as many as fit)
    def probe_encode_traffic_raw(self, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, wpc=-1):
        return _check(lib.fec_probe_encode_traffic(self._h, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, wpc),
                      "fec_probe_encode_traffic")

    def probe_recover_traffic_raw(self, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, masks, out, out_bs,
                                  wpc=-1):
        return _check(lib.fec_probe_recover_traffic(self._h, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss,
                                                    masks, out, out_bs, wpc), "fec_probe_recover_traffic")

    def probe_rebuild_traffic_raw(self, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss, masks, out, out_bs,
                                  wpc=-1):
        return _check(lib.fec_probe_rebuild_traffic(self._h, k, m, shard_len, nblocks, data, dbs, parity, pbs, ss,
                                                    masks, out, out_bs, wpc), "fec_probe_rebuild_traffic")

    def probe_stream_traffic_raw(self, nin, shard_len, nblocks, data, in_bs, out, out_bs, ss, wpc=0):
        return _check(lib.fec_probe_stream_traffic(self._h, nin, shard_len, nblocks, data, in_bs, out, out_bs, ss, wpc),
                      "fec_probe_stream_traffic")

    def probe_link(self, nbytes=512 << 20, reps=3):
        """{h2d, d2h, duplex_each} GB/s of pinned hipMemcpyAsync on this ctx's device."""
        out = (ctypes.c_double * 3)()
        _check(lib.fec_probe_link(self._h, nbytes, reps, out), "fec_probe_link")
        return {"bytes": nbytes, "h2d_GBps": round(out[0], 2), "d2h_GBps": round(out[1], 2),
                "duplex_each_GBps": round(out[2], 2)}

    def xor_encode(self, k, shards, shard_len=None):
        B, n, S = _shape3(shards)
        assert n == k + 1
        a, kind = _addr(shards)
        L = S if shard_len is None else shard_len
        return _check(lib.fec_xor_encode_batch(self._h, k, L, B, a, n * S, a + k * S, n * S, S, kind),
                      "fec_xor_encode_batch")

    def xor_reconstruct(self, k, shards, masks, status=None, shard_len=None):
        B, n, S = _shape3(shards)
        assert n == k + 1
        a, kind = _addr(shards)
        fn = lambda B_, L, d, dbs, p, pbs, ss, ma, sa, kd: lib.fec_xor_reconstruct_batch(
            self._h, k, L, B_, d, dbs, p, pbs, ss, ma, sa, kd)
        return self._recon(fn, "fec_xor_reconstruct_batch", k, 1, B, S, a, n * S, a + k * S, n * S, kind,
                           masks, status, shard_len)
