"""Wire codecs of the FEC frames (include/fec_wire.h) against the reference's own varint test
vectors (quicvarint/varint_test.go:21-110) and the frame layouts of
internal/wire/fec_{repair,source_symbol}_frame.go. No GPU."""
import importlib

import pytest


@pytest.fixture(scope="module")
def W(fec):
    return importlib.import_module("0xfec_amd.wire")


# quicvarint/varint_test.go:21-58 (decoding) and :64-110 (encoding with minimal length)
READ_VECTORS = [
    (bytes([0b00011001]), 25),
    (bytes([0b01000000, 0x25]), 37),                       # encoded too long, still valid
    (bytes([0b01111011, 0xbd]), 15293),
    (bytes([0b10011101, 0x7f, 0x3e, 0x7d]), 494878333),
    (bytes([0b11000010, 0x19, 0x7c, 0x5e, 0xff, 0x14, 0xe8, 0x8c]), 151288809941952652),
]
APPEND_VECTORS = [
    (37, bytes([0x25])),
    (63, bytes([0b00111111])),
    (64, bytes([0x40, 64])),
    (15293, bytes([0b01000000 ^ 0x3b, 0xbd])),
    (494878333, bytes([0b10000000 ^ 0x1d, 0x7f, 0x3e, 0x7d])),
    (151288809941952652, bytes([0xc2, 0x19, 0x7c, 0x5e, 0xff, 0x14, 0xe8, 0x8c])),
]


@pytest.mark.parametrize("data,value", READ_VECTORS)
def test_varint_read_reference_vectors(W, data, value):
    v, used, err = W.varint_read(data + b"\xff\xff")
    assert err is None and v == value and used == len(data)


@pytest.mark.parametrize("value,data", APPEND_VECTORS)
def test_varint_append_reference_vectors(W, value, data):
    assert W.varint_append(b"", value) == data
    assert W.varint_len(value) == len(data)


def test_varint_limits_and_eof(W):
    for v, n in [(63, 1), (64, 2), (16383, 2), (16384, 4), (1073741823, 4), (1073741824, 8), (W.VARINT_MAX, 8)]:
        assert W.varint_len(v) == n
        assert W.varint_read(W.varint_append(b"", v))[:2] == (v, n)
    assert W.varint_len(W.VARINT_MAX + 1) == 0
    with pytest.raises(ValueError):
        W.varint_append(b"", W.VARINT_MAX + 1)
    assert W.varint_read(b"")[2] == "EOF"
    assert W.varint_read(b"\x40")[2] == "EOF"
    assert W.varint_read(b"\xc0\x00\x00")[2] == "EOF"


def test_frame_types_encode_as_the_reference_does(W):
    # repairFrameType = 0x32a80fec (4-byte varint), sourceSymbolFrameType = 0x32a80fec55 (8-byte)
    assert W.varint_append(b"", W.REPAIR_FRAME_TYPE) == bytes([0xb2, 0xa8, 0x0f, 0xec])
    assert W.varint_append(b"", W.SOURCE_SYMBOL_FRAME_TYPE) == bytes([0xc0, 0, 0, 0x32, 0xa8, 0x0f, 0xec, 0x55])


def test_repair_frame_layout_and_round_trip(W):
    f = W.repair_frame_append(b"\x01", 2, 5, b"abc")   # appends to existing bytes
    assert f == b"\x01" + bytes([0xb2, 0xa8, 0x0f, 0xec, 0x02, 0x05, 0x03]) + b"abc"
    assert W.repair_frame_length(2, 5, 3) == len(f) - 1
    body = f[1 + 4:]                                   # the parser has consumed the type
    (bid, pid, payload), used, err = W.parse_repair_frame(body + b"trailing")
    assert err is None and (bid, pid, payload, used) == (2, 5, b"abc", len(body))
    big = bytes(range(256)) * 6
    f = W.repair_frame_append(b"", 1 << 40, 16383, big)
    (bid, pid, payload), used, err = W.parse_repair_frame(f[4:])
    assert (bid, pid, payload, used) == (1 << 40, 16383, big, len(f) - 4)
    assert W.repair_frame_length(1 << 40, 16383, len(big)) == len(f)


def test_repair_frame_parse_errors(W):
    body = W.repair_frame_append(b"", 7, 1, b"\x09" * 10)[4:]
    for cut in range(len(body)):                       # every truncation is io.EOF
        _, _, err = W.parse_repair_frame(body[:cut])
        assert err == "EOF", cut
    (bid, pid, payload), used, err = W.parse_repair_frame(bytes([0x07, 0x01, 0x00]))
    assert err is None and payload is None and used == 3   # zero length: Payload stays nil


def test_source_symbol_frame_layout_and_round_trip(W):
    payload = b"\x10" * 1200
    f = W.source_symbol_frame_append(b"", 300, payload)
    hdr = W.source_symbol_frame_header_len(300, len(payload))
    assert hdr == 8 + 2 + 2 and W.source_symbol_frame_length(300, len(payload)) == len(f) == hdr + 1200
    assert f[:8] == bytes([0xc0, 0, 0, 0x32, 0xa8, 0x0f, 0xec, 0x55])
    (ssid, p), used, err = W.parse_source_symbol_frame(f[8:])
    assert err is None and ssid == 300 and p == payload and used == len(f) - 8
    for cut in (0, 1, 2, 3, len(f) - 9):
        assert W.parse_source_symbol_frame(f[8:8 + cut])[2] == "EOF"
    (ssid, p), used, err = W.parse_source_symbol_frame(bytes([0x05, 0x00]))
    assert err is None and p is None and used == 2


def test_submit_payloads_checks_before_device_work(W, fec):
    B = importlib.import_module("0xfec_amd.batch")
    S = importlib.import_module("0xfec_amd.scheme")
    enc, err = B.BatchEncoder.new(S.REED_SOLOMON_FEC_SCHEME, 3, 2)
    assert err is None
    q = B.RepairQueue()
    assert W.submit_payloads(enc, 0, [b"a", b"b"], q) == \
        "block does not have enough source symbols to generate repair symbols"
    assert "1435" in W.submit_payloads(enc, 0, [b"a", b"b", b"c" * 1435], q)
