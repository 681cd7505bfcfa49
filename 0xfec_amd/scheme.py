"""Python face of the host-side mirror of internal/fec (include/fec_scheme.h).

Names and return conventions follow the reference's Go API so that tests read like
internal/fec/*_test.go: methods return (result, err) where err is the Go error text or None,
and a nil result is None.

    b = Block.literal(id=2, tot_src=20, tot_rep=10, biggest=1434, smallest=20, largest=39)
    b.put_source(20, payload, cap=1452)
    scheme, err = new_reed_solomon_scheme(20, 10)
    frames, err = scheme.repair_symbols(b)          # [(block_id, parity_id, bytes)]
    payloads, err = scheme.recover_symbol_payloads(b)
"""
import ctypes

from . import lib, FEC_OK

MAX_PACKET_BUFFER_SIZE = 1452       # internal/protocol/protocol.go:111
MAX_FEC_PACKET_BUFFER_SIZE = 1434   # internal/protocol/protocol.go:136-138
REPAIR_PAYLOAD_METADATA_LEN = 2     # internal/protocol/protocol.go:140

FEC_DISABLED, XOR_FEC_SCHEME, REED_SOLOMON_FEC_SCHEME = 0, 1, 2   # internal/protocol/fec.go:21-27
FEC_ERR_SCHEME = -20

_vp, _sz, _i, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
_pp = ctypes.POINTER(ctypes.c_void_p)

lib.fec_last_error.restype = ctypes.c_char_p
lib.fec_block_new.restype = _vp
lib.fec_block_new.argtypes = [_u64, _i, _i]
lib.fec_block_literal.restype = _vp
lib.fec_block_literal.argtypes = [_u64, _i, _i, _i, _u64, _u64]
lib.fec_block_free.argtypes = [_vp]
lib.fec_block_free.restype = None
lib.fec_block_put_source.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz]
lib.fec_block_put_repair.argtypes = [_vp, _u64, ctypes.c_char_p, _sz]
lib.fec_block_add_source_symbol.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz]
lib.fec_block_add_repair_symbol.argtypes = [_vp, _u64, _u64, ctypes.c_char_p, _sz]
for _f in ("fec_block_is_recoverable", "fec_block_is_complete", "fec_block_biggest", "fec_block_num_sources"):
    getattr(lib, _f).argtypes = [_vp]
lib.fec_block_get_source.restype = ctypes.c_long
lib.fec_block_get_source.argtypes = [_vp, _u64, _vp, _sz]
lib.fec_scheme_new.restype = _vp
lib.fec_scheme_new.argtypes = [_i, _i, _i, _i]
lib.fec_scheme_free.argtypes = [_vp]
lib.fec_scheme_free.restype = None
lib.fec_scheme_repair_symbols.argtypes = [_vp, _vp, _pp]
lib.fec_scheme_recover_symbol_payloads.argtypes = [_vp, _vp, _pp]
lib.fec_frames_count.restype = _sz
lib.fec_frames_count.argtypes = [_vp]
lib.fec_frames_get.argtypes = [_vp, _sz, ctypes.POINTER(_u64), ctypes.POINTER(_u64),
                               ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(_sz)]
lib.fec_frames_free.argtypes = [_vp]
lib.fec_frames_free.restype = None
lib.fec_bytes_data.restype = ctypes.POINTER(ctypes.c_uint8)
lib.fec_bytes_data.argtypes = [_vp]
lib.fec_bytes_len.restype = _sz
lib.fec_bytes_len.argtypes = [_vp]
lib.fec_bytes_free.argtypes = [_vp]
lib.fec_bytes_free.restype = None
for _f in ("fec_manager_new_sender", "fec_manager_new_receiver"):
    getattr(lib, _f).restype = _vp
    getattr(lib, _f).argtypes = [_i, _i, ctypes.POINTER(_i)]
lib.fec_manager_new.restype = _vp
lib.fec_manager_new.argtypes = [_i, _i, _i, _i, ctypes.POINTER(_i)]
lib.fec_manager_free.argtypes = [_vp]
lib.fec_manager_free.restype = None
lib.fec_manager_next_ssid.restype = _u64
lib.fec_manager_next_ssid.argtypes = [_vp]
lib.fec_manager_block_id.restype = _u64
lib.fec_manager_block_id.argtypes = [_vp, _u64]
lib.fec_manager_add_source_symbol_frame.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz, _pp]
lib.fec_manager_handle_repair_frame.argtypes = [_vp, _u64, _u64, ctypes.c_char_p, _sz, _pp]
lib.fec_manager_handle_source_symbol_frame.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz, _pp]
lib.fec_manager_set_recover_on_source.argtypes = [_vp, _i]
lib.fec_manager_handle_source_symbol_frame_recover.argtypes = [_vp, _u64, ctypes.c_char_p, _sz, _sz, _pp, _pp]


def _err(rc):
    if rc == FEC_OK:
        return None
    return lib.fec_last_error().decode() or ("error %d" % rc)


def _frames(h):
    if not h:
        return None
    out = []
    try:
        for i in range(lib.fec_frames_count(h)):
            bid, pid, ln = _u64(), _u64(), _sz()
            p = ctypes.POINTER(ctypes.c_uint8)()
            lib.fec_frames_get(h, i, ctypes.byref(bid), ctypes.byref(pid), ctypes.byref(p), ctypes.byref(ln))
            out.append((bid.value, pid.value, ctypes.string_at(p, ln.value) if ln.value else b""))
    finally:
        lib.fec_frames_free(h)
    return out


def _bytes(h):
    if not h:
        return None
    try:
        n = lib.fec_bytes_len(h)
        return ctypes.string_at(lib.fec_bytes_data(h), n) if n else b""
    finally:
        lib.fec_bytes_free(h)


class Block:
    """internal/fec/block.go:23-95."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def new(cls, id, tot_src, tot_rep):
        return cls(lib.fec_block_new(id, tot_src, tot_rep))

    @classmethod
    def literal(cls, id=0, tot_src=0, tot_rep=0, biggest=0, smallest=0, largest=0, sources=None, repairs=None):
        b = cls(lib.fec_block_literal(id, tot_src, tot_rep, biggest, smallest, largest))
        for ssid, (data, cap) in (sources or {}).items():
            b.put_source(ssid, data, cap)
        for pid, data in (repairs or {}).items():
            b.put_repair(pid, data)
        return b

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_block_free(self._h)
            self._h = None

    def put_source(self, ssid, data, cap=None):
        data = bytes(data)
        lib.fec_block_put_source(self._h, ssid, data, len(data), len(data) if cap is None else cap)

    def put_repair(self, pid, data):
        data = bytes(data)
        lib.fec_block_put_repair(self._h, pid, data, len(data))

    def add_source_symbol(self, ssid, data, cap=MAX_PACKET_BUFFER_SIZE):
        data = bytes(data)
        return _err(lib.fec_block_add_source_symbol(self._h, ssid, data, len(data), cap))

    def add_repair_symbol(self, block_id, pid, data):
        data = bytes(data)
        return _err(lib.fec_block_add_repair_symbol(self._h, block_id, pid, data, len(data)))

    def is_recoverable(self):
        return bool(lib.fec_block_is_recoverable(self._h))

    def is_complete(self):
        return bool(lib.fec_block_is_complete(self._h))

    @property
    def biggest(self):
        return lib.fec_block_biggest(self._h)

    @property
    def num_sources(self):
        return lib.fec_block_num_sources(self._h)

    def get_source(self, ssid):
        n = lib.fec_block_get_source(self._h, ssid, None, 0)
        if n < 0:
            return None
        buf = ctypes.create_string_buffer(max(n, 1))
        lib.fec_block_get_source(self._h, ssid, ctypes.cast(buf, _vp), n)
        return buf.raw[:n]


class _Scheme:
    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_scheme_free(self._h)
            self._h = None

    def repair_symbols(self, block):
        out = _vp()
        rc = lib.fec_scheme_repair_symbols(self._h, block._h, ctypes.byref(out))
        return (_frames(out.value) if rc == FEC_OK else None), _err(rc)

    def recover_symbol_payloads(self, block):
        out = _vp()
        rc = lib.fec_scheme_recover_symbol_payloads(self._h, block._h, ctypes.byref(out))
        return (_bytes(out.value) if rc == FEC_OK else None), _err(rc)


def new_reed_solomon_scheme(k, m, device=0):
    """NewReedSolomonScheme (internal/fec/reed_solomon.go:15-23) -> (scheme, err)."""
    h = lib.fec_scheme_new(REED_SOLOMON_FEC_SCHEME, k, m, device)
    return (_Scheme(h), None) if h else (None, lib.fec_last_error().decode())


def xor_scheme(device=0):
    """xorScheme{} (internal/fec/xor.go:10-12)."""
    return _Scheme(lib.fec_scheme_new(XOR_FEC_SCHEME, 0, 0, device))


class Manager:
    """internal/fec/manager.go:41-227."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        if getattr(self, "_h", None):
            lib.fec_manager_free(self._h)
            self._h = None

    def next_ssid(self):
        return lib.fec_manager_next_ssid(self._h)

    def block_id(self, ssid):
        return lib.fec_manager_block_id(self._h, ssid)

    def add_source_symbol_frame(self, ssid, payload, cap=MAX_PACKET_BUFFER_SIZE):
        payload = bytes(payload)
        out = _vp()
        rc = lib.fec_manager_add_source_symbol_frame(self._h, ssid, payload, len(payload), cap, ctypes.byref(out))
        return (_frames(out.value) if rc == FEC_OK else None), _err(rc)

    def handle_repair_frame(self, block_id, parity_id, payload):
        payload = bytes(payload)
        out = _vp()
        rc = lib.fec_manager_handle_repair_frame(self._h, block_id, parity_id, payload, len(payload),
                                                 ctypes.byref(out))
        return (_bytes(out.value) if rc == FEC_OK else None), _err(rc)

    def handle_source_symbol_frame(self, ssid, payload, cap=MAX_PACKET_BUFFER_SIZE):
        payload = bytes(payload)
        out = _vp()
        rc = lib.fec_manager_handle_source_symbol_frame(self._h, ssid, payload, len(payload), cap,
                                                        ctypes.byref(out))
        return (_bytes(out.value) if rc == FEC_OK else None), _err(rc)

    def set_recover_on_source(self, on=True):
        """Extension (default off): also recover when a SOURCE symbol makes a block recoverable;
        the reference recovers only on a REPAIR arrival (manager.go:181 vs :221-226)."""
        lib.fec_manager_set_recover_on_source(self._h, 1 if on else 0)

    def handle_source_symbol_frame_recover(self, ssid, payload, cap=MAX_PACKET_BUFFER_SIZE):
        """HandleSourceSymbolFrame plus what it recovered -> (payload, recovered | None, err)."""
        payload = bytes(payload)
        out, rec = _vp(), _vp()
        rc = lib.fec_manager_handle_source_symbol_frame_recover(self._h, ssid, payload, len(payload), cap,
                                                                ctypes.byref(out), ctypes.byref(rec))
        if rc != FEC_OK:
            return None, None, _err(rc)
        return _bytes(out.value), _bytes(rec.value), None


def _mk(fn, *args):
    err = _i(0)
    h = fn(*args, ctypes.byref(err))
    if err.value != FEC_OK:
        return None, lib.fec_last_error().decode()
    return (Manager(h) if h else None), None


def new_sender(scheme_id, device=0):
    """NewSender (manager.go:50-71) -> (manager | None, err)."""
    return _mk(lib.fec_manager_new_sender, scheme_id, device)


def new_receiver(scheme_id, device=0):
    """NewReceiver (manager.go:73-94) -> (manager | None, err)."""
    return _mk(lib.fec_manager_new_receiver, scheme_id, device)


def new_manager(scheme_id, k, m, device=0):
    """NewManager (manager.go:96-109) over a fresh scheme -> (manager | None, err)."""
    return _mk(lib.fec_manager_new, scheme_id, k, m, device)
