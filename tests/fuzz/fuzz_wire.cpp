// fuzz_wire.cpp — libFuzzer target for the FEC frame parsers (include/fec_wire.h).
//
// Each input is parsed by fec_repair_frame_parse and fec_source_symbol_frame_parse and by an
// independent byte-at-a-time model of the reference's parsers (a bytes.Reader fed to
// quicvarint.Read, varint.go:24-71, then the payload-length check and io.ReadFull of
// fec_repair_frame.go:16-42 / fec_source_symbol_frame.go:19-41). Checked on every input:
//   * the result is OK or FEC_ERR_EOF (io.EOF), nothing else, exactly when the model says so;
//   * consumed = the reader position the reference is left at (ReadByte consumes what it read
//     before failing; a too-long payload length leaves the reader after the varints);
//   * on success the fields, payload offset and length equal the model's, and re-encoding the
//     parsed frame (Append, minimal varints) parses back to the same fields and payload.
// Built with -fsanitize=fuzzer,address,undefined (tests/c/build.py); the CPU test runs it for a
// bounded number of inputs from a seed corpus of valid frames and truncations.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "fec_hip.h"
#include "fec_wire.h"

namespace {

struct Model {   // bytes.Reader
    const uint8_t* p;
    size_t n, pos = 0;
    bool readByte(uint8_t* b) {
        if (pos >= n) return false;
        *b = p[pos++];
        return true;
    }
    // quicvarint.Read: one ReadByte per byte, returns at the first failure
    bool varint(uint64_t* v) {
        uint8_t b;
        if (!readByte(&b)) return false;
        const int len = 1 << ((b & 0xc0) >> 6);
        uint64_t x = b & 0x3f;
        for (int i = 1; i < len; ++i) {
            if (!readByte(&b)) return false;
            x = (x << 8) | b;
        }
        *v = x;
        return true;
    }
};

struct Parsed {
    int rc;
    uint64_t a, b;
    size_t off, len, consumed;
};

Parsed model_parse(const uint8_t* d, size_t n, int nids) {
    Model r{d, n};
    Parsed o{FEC_OK, 0, 0, 0, 0, 0};
    uint64_t ids[2] = {0, 0}, plen = 0;
    for (int i = 0; i < nids; ++i)
        if (!r.varint(&ids[i])) return Parsed{FEC_ERR_EOF, 0, 0, 0, 0, r.pos};
    if (!r.varint(&plen)) return Parsed{FEC_ERR_EOF, 0, 0, 0, 0, r.pos};
#ifdef FUZZ_MUTANT   // self-test build (tests/test_sanitizers.py): a model off by one must be caught
    if (plen >= (uint64_t)(r.n - r.pos) && plen) return Parsed{FEC_ERR_EOF, 0, 0, 0, 0, r.pos};
#endif
    if (plen > (uint64_t)(r.n - r.pos)) return Parsed{FEC_ERR_EOF, 0, 0, 0, 0, r.pos};
    o.a = ids[0];
    o.b = ids[1];
    o.off = r.pos;
    o.len = (size_t)plen;
    o.consumed = r.pos + (size_t)plen;
    return o;
}

void check(bool ok) {
    if (!ok) abort();
}

void repair(const uint8_t* d, size_t n) {
    uint64_t bid = 0, pid = 0;
    size_t off = 0, len = 0, consumed = 0;
    const int rc = fec_repair_frame_parse(d, n, &bid, &pid, &off, &len, &consumed);
    const Parsed m = model_parse(d, n, 2);
    check(rc == m.rc && consumed == m.consumed && consumed <= n);
    if (rc != FEC_OK) return;
    check(bid == m.a && pid == m.b && off == m.off && len == m.len && off + len == consumed);
    // Append(parsed) parses back to itself; the frame type comes first on the wire
    const size_t total = fec_repair_frame_length(bid, pid, len);
    std::vector<uint8_t> w(total);
    check(fec_repair_frame_append(w.data(), total, bid, pid, d + off, len) == total);
    uint64_t t = 0;
    size_t tc = 0;
    check(fec_varint_read(w.data(), total, &t, &tc) == FEC_OK && t == FEC_WIRE_REPAIR_FRAME_TYPE);
    uint64_t bid2, pid2;
    size_t off2, len2, c2;
    check(fec_repair_frame_parse(w.data() + tc, total - tc, &bid2, &pid2, &off2, &len2, &c2) == FEC_OK);
    check(bid2 == bid && pid2 == pid && len2 == len && c2 == total - tc &&
          (len == 0 || memcmp(w.data() + tc + off2, d + off, len) == 0));
    check(fec_repair_frame_append(w.data(), total - 1, bid, pid, d + off, len) == 0);   // too small: nothing
}

void source(const uint8_t* d, size_t n) {
    uint64_t ssid = 0;
    size_t off = 0, len = 0, consumed = 0;
    const int rc = fec_source_symbol_frame_parse(d, n, &ssid, &off, &len, &consumed);
    const Parsed m = model_parse(d, n, 1);
    check(rc == m.rc && consumed == m.consumed && consumed <= n);
    if (rc != FEC_OK) return;
    check(ssid == m.a && off == m.off && len == m.len && off + len == consumed);
    const size_t total = fec_source_symbol_frame_length(ssid, len);
    check(total == fec_source_symbol_frame_header_len(ssid, len) + len);
    std::vector<uint8_t> w(total);
    check(fec_source_symbol_frame_append(w.data(), total, ssid, d + off, len) == total);
    uint64_t t = 0;
    size_t tc = 0;
    check(fec_varint_read(w.data(), total, &t, &tc) == FEC_OK && t == FEC_WIRE_SOURCE_SYMBOL_FRAME_TYPE);
    uint64_t s2;
    size_t off2, len2, c2;
    check(fec_source_symbol_frame_parse(w.data() + tc, total - tc, &s2, &off2, &len2, &c2) == FEC_OK);
    check(s2 == ssid && len2 == len && c2 == total - tc && (len == 0 || memcmp(w.data() + tc + off2, d + off, len) == 0));
}

void varint(const uint8_t* d, size_t n) {
    uint64_t v = 0;
    size_t c = 0;
    const int rc = fec_varint_read(d, n, &v, &c);
    Model r{d, n};
    uint64_t mv = 0;
    const bool ok = r.varint(&mv);
    check((rc == FEC_OK) == ok && c == r.pos);
    if (!ok) return;
    check(v == mv && v <= FEC_WIRE_VARINT_MAX);
    uint8_t w[8];
    const size_t l = fec_varint_append(w, sizeof w, v);   // minimal re-encoding
    check(l == fec_varint_len(v) && l <= c);
    uint64_t v2 = 0;
    size_t c2 = 0;
    check(fec_varint_read(w, l, &v2, &c2) == FEC_OK && v2 == v && c2 == l);
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
    // a copy of exactly `size` bytes, so any read past the end is an ASan report
    uint8_t* d = size ? (uint8_t*)malloc(size) : nullptr;
    if (size) memcpy(d, data, size);
    repair(d, size);
    source(d, size);
    varint(d, size);
    free(d);
    return 0;
}
