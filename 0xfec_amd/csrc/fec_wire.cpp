// fec_wire.cpp — QUIC varints and the FEC frames' wire codecs (include/fec_wire.h), restated
// from quicvarint/varint.go and internal/wire/fec_{repair,source_symbol}_frame.go.
#include "../../include/fec_wire.h"

#include <string.h>

#include "../../include/fec_hip.h"

namespace {

constexpr uint64_t kMax1 = 63, kMax2 = 16383, kMax4 = 1073741823, kMax8 = FEC_WIRE_VARINT_MAX;   // varint.go:18-21

struct Reader {   // bytes.Reader over [p, p+n)
    const uint8_t* p;
    size_t n, off = 0;
    int varint(uint64_t* v) {   // quicvarint.Read (varint.go:25-71)
        if (off >= n) return FEC_ERR_EOF;
        const uint8_t first = p[off];
        const size_t len = (size_t)1 << ((first & 0xC0) >> 6);
        if (n - off < len) {
            off = n;   // the reference consumes what it read before failing
            return FEC_ERR_EOF;
        }
        uint64_t x = first & 0x3F;
        for (size_t i = 1; i < len; ++i) x = (x << 8) | p[off + i];
        off += len;
        *v = x;
        return FEC_OK;
    }
};

}  // namespace

extern "C" {

size_t fec_varint_len(uint64_t v) {   // varint.go:122-138
    return v <= kMax1 ? 1 : v <= kMax2 ? 2 : v <= kMax4 ? 4 : v <= kMax8 ? 8 : 0;
}

size_t fec_varint_append(uint8_t* dst, size_t cap, uint64_t v) {   // varint.go:74-91
    const size_t len = fec_varint_len(v);
    if (!len || !dst || cap < len) return 0;
    const uint8_t prefix = len == 1 ? 0x00 : len == 2 ? 0x40 : len == 4 ? 0x80 : 0xC0;
    for (size_t i = 0; i < len; ++i) dst[i] = (uint8_t)(v >> (8 * (len - 1 - i)));
    dst[0] |= prefix;
    return len;
}

int fec_varint_read(const uint8_t* src, size_t len, uint64_t* v, size_t* consumed) {
    if (!src && len) return FEC_ERR_INVALID_ARG;
    Reader r{src, len};
    uint64_t x = 0;
    const int rc = r.varint(&x);
    if (consumed) *consumed = r.off;
    if (rc == FEC_OK && v) *v = x;
    return rc;
}

size_t fec_repair_frame_length(uint64_t block_id, uint64_t parity_id, size_t payload_len) {
    // fec_repair_frame.go:55-57
    return fec_varint_len(FEC_WIRE_REPAIR_FRAME_TYPE) + fec_varint_len(block_id) + fec_varint_len(parity_id) +
           fec_varint_len(payload_len) + payload_len;
}

size_t fec_repair_frame_append(uint8_t* dst, size_t cap, uint64_t block_id, uint64_t parity_id, const uint8_t* payload,
                               size_t len) {   // fec_repair_frame.go:45-52
    const size_t total = fec_repair_frame_length(block_id, parity_id, len);
    if (!dst || cap < total || (len && !payload) || !fec_varint_len(block_id) || !fec_varint_len(parity_id)) return 0;
    size_t o = 0;
    o += fec_varint_append(dst + o, cap - o, FEC_WIRE_REPAIR_FRAME_TYPE);
    o += fec_varint_append(dst + o, cap - o, block_id);
    o += fec_varint_append(dst + o, cap - o, parity_id);
    o += fec_varint_append(dst + o, cap - o, len);
    if (len) memcpy(dst + o, payload, len);
    return o + len;
}

int fec_repair_frame_parse(const uint8_t* src, size_t len, uint64_t* block_id, uint64_t* parity_id, size_t* payload_off,
                           size_t* payload_len, size_t* consumed) {   // fec_repair_frame.go:16-42
    if (!src && len) return FEC_ERR_INVALID_ARG;
    Reader r{src, len};
    uint64_t bid = 0, pid = 0, plen = 0;
    int rc;
    if ((rc = r.varint(&bid)) || (rc = r.varint(&pid)) || (rc = r.varint(&plen))) {
        if (consumed) *consumed = r.off;
        return rc;
    }
    if (plen > r.n - r.off) {   // payloadLen > r.Len() -> io.EOF
        if (consumed) *consumed = r.off;
        return FEC_ERR_EOF;
    }
    if (block_id) *block_id = bid;
    if (parity_id) *parity_id = pid;
    if (payload_off) *payload_off = r.off;
    if (payload_len) *payload_len = (size_t)plen;   // 0: the reference leaves Payload nil
    if (consumed) *consumed = r.off + (size_t)plen;
    return FEC_OK;
}

size_t fec_source_symbol_frame_header_len(uint64_t ssid, size_t payload_len) {   // fec_source_symbol_frame.go:43-45
    return fec_varint_len(FEC_WIRE_SOURCE_SYMBOL_FRAME_TYPE) + fec_varint_len(ssid) + fec_varint_len(payload_len);
}

size_t fec_source_symbol_frame_length(uint64_t ssid, size_t payload_len) {   // fec_source_symbol_frame.go:56-58
    return fec_source_symbol_frame_header_len(ssid, payload_len) + payload_len;
}

size_t fec_source_symbol_frame_append(uint8_t* dst, size_t cap, uint64_t ssid, const uint8_t* payload, size_t len) {
    // fec_source_symbol_frame.go:47-53
    const size_t total = fec_source_symbol_frame_length(ssid, len);
    if (!dst || cap < total || (len && !payload) || !fec_varint_len(ssid)) return 0;
    size_t o = 0;
    o += fec_varint_append(dst + o, cap - o, FEC_WIRE_SOURCE_SYMBOL_FRAME_TYPE);
    o += fec_varint_append(dst + o, cap - o, ssid);
    o += fec_varint_append(dst + o, cap - o, len);
    if (len) memcpy(dst + o, payload, len);
    return o + len;
}

int fec_source_symbol_frame_parse(const uint8_t* src, size_t len, uint64_t* ssid, size_t* payload_off,
                                  size_t* payload_len, size_t* consumed) {   // fec_source_symbol_frame.go:19-41
    if (!src && len) return FEC_ERR_INVALID_ARG;
    Reader r{src, len};
    uint64_t sid = 0, plen = 0;
    int rc;
    if ((rc = r.varint(&sid)) || (rc = r.varint(&plen))) {
        if (consumed) *consumed = r.off;
        return rc;
    }
    if (plen > r.n - r.off) {
        if (consumed) *consumed = r.off;
        return FEC_ERR_EOF;
    }
    if (ssid) *ssid = sid;
    if (payload_off) *payload_off = r.off;
    if (payload_len) *payload_len = (size_t)plen;   // the reference copies into make(len, 1452)
    if (consumed) *consumed = r.off + (size_t)plen;
    return FEC_OK;
}

}  // extern "C"
