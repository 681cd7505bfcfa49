"""Python face of the sender-side batching layer (include/fec_batch.h, fec_batch.hpp).

    q = RepairQueue()                         # repair_queue.go: Add / Peek / Pop, 32 frames
    enc, err = BatchEncoder.new(REED_SOLOMON_FEC_SCHEME, 20, 10, max_blocks=1024)
    err = sender.add_source_symbol_frame_batched(ssid, payload, enc, q)   # defers the encode
    n, err = enc.drain()                      # one H2D + launch + D2H for every staged block
    q.peek() -> (block_id, parity_id, payload) | None ; q.pop()
"""
import ctypes

from . import lib, FEC_OK
from .scheme import MAX_PACKET_BUFFER_SIZE, Manager, _bytes, _err

_vp, _sz, _i, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64

lib.fec_repair_queue_new.restype = _vp
lib.fec_repair_queue_new.argtypes = [_sz]
lib.fec_repair_queue_free.argtypes = [_vp]
lib.fec_repair_queue_free.restype = None
lib.fec_repair_queue_add.argtypes = [_vp, _u64, _u64, ctypes.c_char_p, _sz]
lib.fec_repair_queue_peek.argtypes = [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                                      ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(_sz),
                                      ctypes.POINTER(_sz)]
lib.fec_repair_queue_pop.argtypes = [_vp]
lib.fec_repair_queue_pop.restype = None
lib.fec_repair_queue_len.restype = _sz
lib.fec_repair_queue_len.argtypes = [_vp]
lib.fec_repair_queue_has_data_calls.restype = _u64
lib.fec_repair_queue_has_data_calls.argtypes = [_vp]
lib.fec_repair_queue_close.argtypes = [_vp, ctypes.c_char_p]
lib.fec_repair_queue_close.restype = None
lib.fec_batch_encoder_new.restype = _vp
lib.fec_batch_encoder_new.argtypes = [_i, _i, _i, _sz, _i, ctypes.POINTER(_i)]
lib.fec_batch_encoder_free.argtypes = [_vp]
lib.fec_batch_encoder_free.restype = None
lib.fec_batch_encoder_submit.argtypes = [_vp, _vp, _vp]
lib.fec_batch_encoder_flush.argtypes = [_vp]
lib.fec_batch_encoder_poll.argtypes = [_vp, ctypes.POINTER(_sz)]
lib.fec_batch_encoder_drain.argtypes = [_vp, ctypes.POINTER(_sz)]
lib.fec_batch_encoder_staged.restype = _sz
lib.fec_batch_encoder_staged.argtypes = [_vp]
lib.fec_batch_encoder_in_flight.restype = _sz
lib.fec_batch_encoder_in_flight.argtypes = [_vp]
lib.fec_batch_encoder_backlog.restype = _sz
lib.fec_batch_encoder_backlog.argtypes = [_vp]
lib.fec_manager_add_source_symbol_frame_batched.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz, _vp, _vp]
lib.fec_recovered_queue_new.restype = _vp
lib.fec_recovered_queue_new.argtypes = []
lib.fec_recovered_queue_free.argtypes = [_vp]
lib.fec_recovered_queue_free.restype = None
lib.fec_recovered_queue_len.restype = _sz
lib.fec_recovered_queue_len.argtypes = [_vp]
lib.fec_recovered_queue_pop.argtypes = [_vp, ctypes.POINTER(_u64), ctypes.POINTER(_vp)]
lib.fec_batch_decoder_new.restype = _vp
lib.fec_batch_decoder_new.argtypes = [_i, _i, _i, _sz, _i, ctypes.POINTER(_i)]
lib.fec_batch_decoder_free.argtypes = [_vp]
lib.fec_batch_decoder_free.restype = None
lib.fec_batch_decoder_submit.argtypes = [_vp, _vp, _vp, ctypes.POINTER(_i)]
lib.fec_batch_decoder_flush.argtypes = [_vp]
lib.fec_batch_decoder_poll.argtypes = [_vp, ctypes.POINTER(_sz)]
lib.fec_batch_decoder_drain.argtypes = [_vp, ctypes.POINTER(_sz)]
lib.fec_batch_decoder_staged.restype = _sz
lib.fec_batch_decoder_staged.argtypes = [_vp]
lib.fec_batch_decoder_in_flight.restype = _sz
lib.fec_batch_decoder_in_flight.argtypes = [_vp]
lib.fec_manager_handle_repair_frame_batched.argtypes = [_vp, _u64, _u64, ctypes.c_char_p, _sz, _vp, _vp]
lib.fec_manager_handle_source_symbol_frame_batched.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz,
                                                               ctypes.POINTER(_vp), _vp, _vp]


class RepairQueue:
    """repair_queue.go:17-99 (max_len 0 -> maxRepairSendQueueLen = 32)."""

    def __init__(self, max_len=0):
        self._h = lib.fec_repair_queue_new(max_len)

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_repair_queue_free(self._h)
            self._h = None

    def add(self, block_id, parity_id, payload):
        payload = bytes(payload)
        return _err(lib.fec_repair_queue_add(self._h, block_id, parity_id, payload, len(payload)))

    def peek(self):
        bid, pid, ln, cap = _u64(), _u64(), _sz(), _sz()
        p = ctypes.POINTER(ctypes.c_uint8)()
        if not lib.fec_repair_queue_peek(self._h, ctypes.byref(bid), ctypes.byref(pid), ctypes.byref(p),
                                         ctypes.byref(ln), ctypes.byref(cap)):
            return None
        return bid.value, pid.value, (ctypes.string_at(p, ln.value) if ln.value else b"")

    def peek_cap(self):
        cap = _sz()
        if not lib.fec_repair_queue_peek(self._h, None, None, None, None, ctypes.byref(cap)):
            return None
        return cap.value

    def pop(self):
        lib.fec_repair_queue_pop(self._h)

    def __len__(self):
        return lib.fec_repair_queue_len(self._h)

    @property
    def has_data_calls(self):
        return lib.fec_repair_queue_has_data_calls(self._h)

    def close_with_error(self, msg):
        lib.fec_repair_queue_close(self._h, msg.encode())

    def drain_frames(self):
        out = []
        while True:
            f = self.peek()
            if f is None:
                return out
            out.append(f)
            self.pop()


class BatchEncoder:
    """Deferred, batched repairSymbols over many blocks (fec_batch.hpp)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def new(cls, scheme_id, k, m, max_blocks=1024, device=0):
        err = _i(0)
        h = lib.fec_batch_encoder_new(scheme_id, k, m, max_blocks, device, ctypes.byref(err))
        if err.value != FEC_OK:
            return None, lib.fec_last_error().decode()
        return cls(h), None

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_batch_encoder_free(self._h)
            self._h = None

    def submit(self, block, queue):
        return _err(lib.fec_batch_encoder_submit(self._h, block._h, queue._h))

    def flush(self):
        return _err(lib.fec_batch_encoder_flush(self._h))

    def poll(self):
        n = _sz()
        rc = lib.fec_batch_encoder_poll(self._h, ctypes.byref(n))
        return n.value, _err(rc)

    def drain(self):
        n = _sz()
        rc = lib.fec_batch_encoder_drain(self._h, ctypes.byref(n))
        return n.value, _err(rc)

    @property
    def staged(self):
        return lib.fec_batch_encoder_staged(self._h)

    @property
    def in_flight(self):
        return lib.fec_batch_encoder_in_flight(self._h)

    @property
    def backlog(self):
        return lib.fec_batch_encoder_backlog(self._h)


def add_source_symbol_frame_batched(manager, ssid, payload, encoder, queue, cap=MAX_PACKET_BUFFER_SIZE):
    """Manager.AddSourceSymbolFrame (manager.go:123-158) with the encode deferred to `encoder`;
    the block's repair frames reach `queue` when its batch completes. Returns err."""
    payload = bytes(payload)
    return _err(lib.fec_manager_add_source_symbol_frame_batched(manager._h, ssid, payload, len(payload), cap,
                                                                encoder._h, queue._h))


Manager.add_source_symbol_frame_batched = (
    lambda self, ssid, payload, encoder, queue, cap=MAX_PACKET_BUFFER_SIZE:
    add_source_symbol_frame_batched(self, ssid, payload, encoder, queue, cap))


class RecoveredQueue:
    """Recovered payloads of one connection, in the order their blocks became recoverable."""

    def __init__(self):
        self._h = lib.fec_recovered_queue_new()

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_recovered_queue_free(self._h)
            self._h = None

    def __len__(self):
        return lib.fec_recovered_queue_len(self._h)

    def pop(self):
        bid, out = _u64(), _vp()
        if not lib.fec_recovered_queue_pop(self._h, ctypes.byref(bid), ctypes.byref(out)):
            return None
        return bid.value, _bytes(out.value)

    def drain(self):
        out = []
        while True:
            it = self.pop()
            if it is None:
                return out
            out.append(it)


class BatchDecoder:
    """Deferred, batched recoverSymbolPayloads over many blocks (fec_batch.hpp)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def new(cls, scheme_id, k, m, max_blocks=1024, device=0):
        err = _i(0)
        h = lib.fec_batch_decoder_new(scheme_id, k, m, max_blocks, device, ctypes.byref(err))
        if err.value != FEC_OK:
            return None, lib.fec_last_error().decode()
        return cls(h), None

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_batch_decoder_free(self._h)
            self._h = None

    def submit(self, block, queue):
        """-> (staged, err); staged False for an already complete block (nil, nil)."""
        st = _i(0)
        rc = lib.fec_batch_decoder_submit(self._h, block._h, queue._h, ctypes.byref(st))
        return bool(st.value), _err(rc)

    def flush(self):
        return _err(lib.fec_batch_decoder_flush(self._h))

    def poll(self):
        n = _sz()
        rc = lib.fec_batch_decoder_poll(self._h, ctypes.byref(n))
        return n.value, _err(rc)

    def drain(self):
        n = _sz()
        rc = lib.fec_batch_decoder_drain(self._h, ctypes.byref(n))
        return n.value, _err(rc)

    @property
    def staged(self):
        return lib.fec_batch_decoder_staged(self._h)

    @property
    def in_flight(self):
        return lib.fec_batch_decoder_in_flight(self._h)


def handle_repair_frame_batched(manager, block_id, parity_id, payload, decoder, queue):
    """Manager.HandleRepairFrame (manager.go:160-198) with the recovery deferred to `decoder`;
    the recovered payload reaches `queue` when its batch completes. Returns err."""
    payload = bytes(payload)
    return _err(lib.fec_manager_handle_repair_frame_batched(manager._h, block_id, parity_id, payload, len(payload),
                                                            decoder._h, queue._h))


Manager.handle_repair_frame_batched = (
    lambda self, block_id, parity_id, payload, decoder, queue:
    handle_repair_frame_batched(self, block_id, parity_id, payload, decoder, queue))


def handle_source_symbol_frame_batched(manager, ssid, payload, decoder, queue, cap=MAX_PACKET_BUFFER_SIZE):
    """Manager.HandleSourceSymbolFrame (manager.go:200-227) -> (payload, err); with
    set_recover_on_source(True), a source that makes its block recoverable stages the block
    into `decoder` and the recovered payload reaches `queue` when its batch completes."""
    payload = bytes(payload)
    out = _vp()
    rc = lib.fec_manager_handle_source_symbol_frame_batched(manager._h, ssid, payload, len(payload), cap,
                                                            ctypes.byref(out), decoder._h, queue._h)
    return (_bytes(out.value) if rc == FEC_OK else None), _err(rc)


Manager.handle_source_symbol_frame_batched = (
    lambda self, ssid, payload, decoder, queue, cap=MAX_PACKET_BUFFER_SIZE:
    handle_source_symbol_frame_batched(self, ssid, payload, decoder, queue, cap))
