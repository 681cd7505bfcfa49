"""Python face of the FEC frames' wire codecs (include/fec_wire.h): quicvarint and the REPAIR /
SOURCE_SYMBOL frames of internal/wire, plus zero-copy staging of a block's source payloads."""
import ctypes

from . import lib, FEC_OK
from .scheme import _err

_vp, _sz, _i, _u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
_psz, _pu64 = ctypes.POINTER(_sz), ctypes.POINTER(_u64)

REPAIR_FRAME_TYPE = 0x32a80fec           # internal/wire/frame_parser.go:38
SOURCE_SYMBOL_FRAME_TYPE = 0x32a80fec55  # internal/wire/frame_parser.go:39
VARINT_MAX = (1 << 62) - 1
FEC_ERR_EOF = -21

lib.fec_varint_len.restype = _sz
lib.fec_varint_len.argtypes = [_u64]
lib.fec_varint_append.restype = _sz
lib.fec_varint_append.argtypes = [ctypes.c_char_p, _sz, _u64]
lib.fec_varint_read.argtypes = [ctypes.c_char_p, _sz, _pu64, _psz]
lib.fec_repair_frame_length.restype = _sz
lib.fec_repair_frame_length.argtypes = [_u64, _u64, _sz]
lib.fec_repair_frame_append.restype = _sz
lib.fec_repair_frame_append.argtypes = [ctypes.c_char_p, _sz, _u64, _u64, ctypes.c_char_p, _sz]
lib.fec_repair_frame_parse.argtypes = [ctypes.c_char_p, _sz, _pu64, _pu64, _psz, _psz, _psz]
lib.fec_source_symbol_frame_length.restype = _sz
lib.fec_source_symbol_frame_length.argtypes = [_u64, _sz]
lib.fec_source_symbol_frame_header_len.restype = _sz
lib.fec_source_symbol_frame_header_len.argtypes = [_u64, _sz]
lib.fec_source_symbol_frame_append.restype = _sz
lib.fec_source_symbol_frame_append.argtypes = [ctypes.c_char_p, _sz, _u64, ctypes.c_char_p, _sz]
lib.fec_source_symbol_frame_parse.argtypes = [ctypes.c_char_p, _sz, _pu64, _psz, _psz, _psz]
lib.fec_batch_encoder_submit_payloads.argtypes = [_vp, _u64, ctypes.POINTER(ctypes.c_char_p), _psz, _i, _vp]


def varint_len(v):
    return lib.fec_varint_len(v)


def varint_append(b, v):
    buf = ctypes.create_string_buffer(8)
    n = lib.fec_varint_append(buf, 8, v)
    if not n:
        raise ValueError("%#x doesn't fit into 62 bits" % v)   # quicvarint.Append panics
    return bytes(b) + buf.raw[:n]


def varint_read(data):
    """-> (value, consumed, err)"""
    data = bytes(data)
    v, used = _u64(), _sz()
    rc = lib.fec_varint_read(data, len(data), ctypes.byref(v), ctypes.byref(used))
    return (v.value if rc == FEC_OK else 0), used.value, (None if rc == FEC_OK else "EOF")


def repair_frame_append(b, block_id, parity_id, payload):
    payload = bytes(payload)
    n = lib.fec_repair_frame_length(block_id, parity_id, len(payload))
    buf = ctypes.create_string_buffer(max(n, 1))
    w = lib.fec_repair_frame_append(buf, n, block_id, parity_id, payload, len(payload))
    assert w == n
    return bytes(b) + buf.raw[:n]


def repair_frame_length(block_id, parity_id, payload_len):
    return lib.fec_repair_frame_length(block_id, parity_id, payload_len)


def parse_repair_frame(data):
    """parseRepairFrame after the frame type -> ((block_id, parity_id, payload | None), consumed, err)."""
    data = bytes(data)
    bid, pid, off, ln, used = _u64(), _u64(), _sz(), _sz(), _sz()
    rc = lib.fec_repair_frame_parse(data, len(data), ctypes.byref(bid), ctypes.byref(pid), ctypes.byref(off),
                                    ctypes.byref(ln), ctypes.byref(used))
    if rc != FEC_OK:
        return None, used.value, "EOF"
    payload = data[off.value:off.value + ln.value] if ln.value else None
    return (bid.value, pid.value, payload), used.value, None


def source_symbol_frame_append(b, ssid, payload):
    payload = bytes(payload)
    n = lib.fec_source_symbol_frame_length(ssid, len(payload))
    buf = ctypes.create_string_buffer(max(n, 1))
    w = lib.fec_source_symbol_frame_append(buf, n, ssid, payload, len(payload))
    assert w == n
    return bytes(b) + buf.raw[:n]


def source_symbol_frame_length(ssid, payload_len):
    return lib.fec_source_symbol_frame_length(ssid, payload_len)


def source_symbol_frame_header_len(ssid, payload_len):
    return lib.fec_source_symbol_frame_header_len(ssid, payload_len)


def parse_source_symbol_frame(data):
    """ParseSourceSymbolFrame after the frame type -> ((ssid, payload | None), consumed, err)."""
    data = bytes(data)
    sid, off, ln, used = _u64(), _sz(), _sz(), _sz()
    rc = lib.fec_source_symbol_frame_parse(data, len(data), ctypes.byref(sid), ctypes.byref(off), ctypes.byref(ln),
                                           ctypes.byref(used))
    if rc != FEC_OK:
        return None, used.value, "EOF"
    payload = data[off.value:off.value + ln.value] if ln.value else None
    return (sid.value, payload), used.value, None


def submit_payloads(encoder, block_id, payloads, queue):
    """Stage a complete block's source payloads (SSID order) straight into pinned staging."""
    payloads = [bytes(p) for p in payloads]
    arr = (ctypes.c_char_p * max(len(payloads), 1))(*payloads)
    lens = (_sz * max(len(payloads), 1))(*[len(p) for p in payloads])
    return _err(lib.fec_batch_encoder_submit_payloads(encoder._h, block_id, arr, lens, len(payloads), queue._h))
