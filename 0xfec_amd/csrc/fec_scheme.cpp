// fec_scheme.cpp — C++ mirror of internal/fec (block.go, reed_solomon.go, xor.go,
// manager.go) over the HIP codec, plus the C ABI of include/fec_scheme.h.
//
// Every function cites the reference lines it restates. Where the Go code would panic
// (index or slice out of range on malformed input), this mirror returns an error instead;
// those cases are listed in DESIGN.md ("Divergences").
#include "../../include/fec_scheme.hpp"

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>

#include "../../include/fec_batch.h"
#include "../../include/fec_batch.hpp"
#include "../../include/fec_hip.h"
#include "../../include/fec_scheme.h"
#include "../../include/fec_wire.h"

namespace fec {

static std::string fmt(const char* f, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, f);
    vsnprintf(buf, sizeof(buf), f, ap);
    va_end(ap);
    return buf;
}

static Error codec_error(int rc) {
    Error e;
    e.code = rc;
    e.msg = fec_strerror(rc);
    return e;
}

// ------------------------------------------------------------------ Slice

Slice Slice::make(size_t len, size_t cap) {
    Slice s;
    s.buf = std::make_shared<std::vector<uint8_t>>(std::max(len, cap), 0);
    s.len = len;
    s.cap = std::max(len, cap);
    return s;
}

Slice Slice::from(const uint8_t* p, size_t len, size_t cap) {
    Slice s = make(len, cap);
    if (len) memcpy(s.data(), p, len);
    return s;
}

Slice Slice::reslice(size_t lo, size_t hi) const {
    Slice s = *this;
    s.off = off + lo;
    s.len = hi - lo;
    s.cap = cap - lo;
    return s;
}

// ------------------------------------------------------------------ Block (block.go)

Block Block::New(BlockID id, int totNumSourceSymbols, int totNumRepairSymbols) {   // block.go:36-49
    Block b;
    b.id = id;
    b.smallestSSID = (SourceSymbolID)id * (SourceSymbolID)totNumSourceSymbols;
    b.largestSSID = b.smallestSSID + (SourceSymbolID)totNumSourceSymbols - 1;
    b.totNumSourceSymbols = (int)((int64_t)b.largestSSID - (int64_t)b.smallestSSID + 1);
    b.totNumRepairSymbols = totNumRepairSymbols;
    b.biggestSourceSymbolLenSoFar = 0;
    return b;
}

Error Block::addSourceSymbol(const SourceSymbolFrame& f) {   // block.go:56-70
    if (f.ssid < smallestSSID || f.ssid > largestSSID)
        return Error::text(fmt("source symbol was provided to the wrong block. Expecting SID within the range "
                               "[%llu, %llu] and got %llu",
                               (unsigned long long)smallestSSID, (unsigned long long)largestSSID,
                               (unsigned long long)f.ssid));
    if (!ssidToSourcePayload.count(f.ssid)) {
        ssidToSourcePayload[f.ssid] = f.payload;
        if (biggestSourceSymbolLenSoFar < (int)f.payload.len) biggestSourceSymbolLenSoFar = (int)f.payload.len;
    }
    return Error::nil();
}

Error Block::addRepairSymbol(const RepairFrame& f) {   // block.go:73-85
    if (id != f.block_id)
        return Error::text(fmt("the repair symbol was provided to the wrong block. Expecting %llu and got %llu",
                               (unsigned long long)id, (unsigned long long)f.block_id));
    if (!pidToRepairPayload.count(f.parity_id)) {
        pidToRepairPayload[f.parity_id] = f.payload;
        biggestSourceSymbolLenSoFar = (int)f.payload.len - (int)kRepairPayloadMetadataLen;
    }
    return Error::nil();
}

bool Block::isRecoverable() const {   // block.go:88-90
    return (int)(ssidToSourcePayload.size() + pidToRepairPayload.size()) >= totNumSourceSymbols;
}

bool Block::isComplete() const {   // block.go:93-95
    return (int)ssidToSourcePayload.size() == totNumSourceSymbols;
}

// ------------------------------------------------------------------ Engine

Engine::~Engine() {
    if (ctx_) fec_ctx_destroy(ctx_);
}

Error Engine::ctx(fec_ctx** out) {
    if (!ctx_) {
        const int rc = fec_ctx_create(device_, &ctx_);
        if (rc) {
            ctx_ = nullptr;
            return codec_error(rc);
        }
    }
    *out = ctx_;
    return Error::nil();
}

// ------------------------------------------------------------------ Reed-Solomon (reed_solomon.go)

static const char* kIncomplete = "block does not have enough source symbols to generate repair symbols";
static const char* kNotRecoverable = "not enough present symbols to repair the missing ones";

Error errIncomplete() { return Error::text(kIncomplete); }

static Error too_big(int biggest) {
    return Error::text(fmt("source symbol payload len is greater is too big for FEC headers. Max %d and got %d",
                           (int)kMaxFECPacketBufferSize, biggest));
}

Error ReedSolomonScheme::New(int k, int m, std::shared_ptr<Engine> engine, std::unique_ptr<ReedSolomonScheme>* out) {
    // reed_solomon.go:15-23 -> reedsolomon.New(k, m) validation
    if (k <= 0 || m < 0) return codec_error(FEC_ERR_INV_SHARD_NUM);
    if (k + m > 256) return codec_error(FEC_ERR_MAX_SHARD_NUM);
    out->reset(new ReedSolomonScheme(k, m, std::move(engine)));
    return Error::nil();
}

Error ReedSolomonScheme::addLengthToSourceSymbolPayload(Block& b, SourceSymbolID ssid, Slice* out) {
    // reed_solomon.go:70-89
    auto it = b.ssidToSourcePayload.find(ssid);
    if (it == b.ssidToSourcePayload.end())
        return Error::text(fmt("block [%llu, %llu] is complete but SID %llu does not exist",
                               (unsigned long long)b.smallestSSID, (unsigned long long)b.largestSSID,
                               (unsigned long long)ssid));
    Slice& payload = it->second;
    const uint16_t payloadLen = (uint16_t)payload.len;
    const int shardLen = (int)kRepairPayloadMetadataLen + b.biggestSourceSymbolLenSoFar;
    if (shardLen > (int)payload.cap)
        return Error::text(fmt("shard len (%d) is greater than capacity of payload (%d)", shardLen, (int)payload.cap));
    if (shardLen < (int)kRepairPayloadMetadataLen)   // Go: negative slice bound panics
        return Error::text(fmt("shard len (%d) is negative", shardLen - 2));
    Slice shard = payload.reslice(0, (size_t)shardLen);
    shard.data()[b.biggestSourceSymbolLenSoFar] = (uint8_t)(payloadLen >> 8);
    shard.data()[b.biggestSourceSymbolLenSoFar + 1] = (uint8_t)(payloadLen & 0xFF);
    *out = shard;
    return Error::nil();
}

Error errTooBig(int biggest) { return too_big(biggest); }

Error ReedSolomonScheme::stageRepairInput(Block& b, uint8_t* dst, size_t stride, size_t* shard_len) {
    // reed_solomon.go:26-51, up to the enc.Encode call: the same checks in the same order
    if (!b.isComplete()) return Error::text(kIncomplete);
    if (b.biggestSourceSymbolLenSoFar > (int)kMaxFECPacketBufferSize) return too_big(b.biggestSourceSymbolLenSoFar);
    const size_t L = kRepairPayloadMetadataLen + (size_t)b.biggestSourceSymbolLenSoFar;
    for (int i = 0; i < b.totNumSourceSymbols; ++i) {
        Slice shard;
        Error e = addLengthToSourceSymbolPayload(b, b.smallestSSID + (SourceSymbolID)i, &shard);
        if (!e.ok()) return e;
        if (i < k_) {
            if (L > stride) return Error::text(fmt("shard len (%zu) exceeds the staging slot (%zu)", L, stride));
            memcpy(dst + (size_t)i * stride, shard.data(), L);
            memset(dst + (size_t)i * stride + L, 0, std::min(stride, (L + 15) & ~(size_t)15) - L);
        }
    }
    // enc.Encode(shards): klauspost checks the shard count, then encodes shards[k:] from shards[:k]
    if (b.totNumSourceSymbols + b.totNumRepairSymbols != k_ + m_)
        return Error::text(std::string("unable to make parity shards: ") + fec_strerror(FEC_ERR_TOO_FEW_SHARDS));
    if (L == 0) return Error::text(std::string("unable to make parity shards: ") + fec_strerror(FEC_ERR_SHARD_NO_DATA));
    *shard_len = L;
    return Error::nil();
}

Error ReedSolomonScheme::repairSymbols(Block& b, std::vector<RepairFrame>* out) {   // reed_solomon.go:26-68
    out->clear();
    const size_t stride = std::max<size_t>(1, kRepairPayloadMetadataLen + (size_t)std::max(0, b.biggestSourceSymbolLenSoFar));
    std::vector<uint8_t> host((size_t)(k_ + m_) * stride);
    size_t L = 0;
    Error e = stageRepairInput(b, host.data(), stride, &L);
    if (!e.ok()) return e;
    const int nsh = k_ + m_;
    if (m_ > 0) {
        fec_ctx* ctx = nullptr;
        e = engine_->ctx(&ctx);
        if (!e.ok()) return e;
        const int rc = fec_rs_encode_batch(ctx, k_, m_, L, 1, host.data(), (size_t)nsh * L, host.data() + (size_t)k_ * L,
                                           (size_t)nsh * L, L, FEC_HOST);
        if (rc) return Error{std::string("unable to make parity shards: ") + fec_strerror(rc), rc};
    }
    out->resize(b.totNumRepairSymbols);
    for (int i = 0; i < b.totNumRepairSymbols; ++i) {
        // repair shards: make([]byte, 0, MaxPacketBufferSize)[:L'] (reed_solomon.go:44-49)
        Slice rep = Slice::make(0, kMaxPacketBufferSize).reslice(0, L);
        memcpy(rep.data(), &host[(size_t)(k_ + i) * L], L);
        (*out)[i].block_id = b.id;
        (*out)[i].parity_id = (ParityID)i;
        (*out)[i].payload = rep;
    }
    return Error::nil();
}

Error ReedSolomonScheme::stageRecoverInput(Block& b, uint8_t* dst, size_t stride, RecoverPlan* plan) {
    // reed_solomon.go:92-124, up to the enc.ReconstructData call: the same checks in the same
    // order, then the present shards into dst + i*stride (n slots; absent slots untouched)
    plan->nothing = false;
    plan->missing.clear();
    if (!b.isRecoverable()) return Error::text(kNotRecoverable);
    if (b.isComplete()) {
        plan->nothing = true;   // nil, nil
        return Error::nil();
    }
    const int nsh = b.totNumSourceSymbols + b.totNumRepairSymbols;
    std::vector<Slice> shards(nsh > 0 ? nsh : 0);
    for (int i = 0; i < b.totNumSourceSymbols; ++i) {
        const SourceSymbolID ssid = b.smallestSSID + (SourceSymbolID)i;
        if (!b.ssidToSourcePayload.count(ssid)) {
            plan->missing.push_back(i);
            continue;
        }
        Error e = addLengthToSourceSymbolPayload(b, ssid, &shards[i]);
        if (!e.ok()) return e;
    }
    for (auto& kv : b.pidToRepairPayload) {
        const uint64_t i = (uint64_t)b.totNumSourceSymbols + kv.first;
        if (i >= (uint64_t)nsh)   // Go: index out of range panic
            return Error::text(fmt("parity id %llu out of range for %d repair symbols",
                                   (unsigned long long)kv.first, b.totNumRepairSymbols));
        shards[i] = kv.second;
    }
    // enc.ReconstructData(shards): klauspost shard-count / size / presence checks
    if (nsh != k_ + m_) return codec_error(FEC_ERR_TOO_FEW_SHARDS);
    size_t L = 0;
    for (auto& sh : shards)
        if (!sh.nil() && sh.len) { L = sh.len; break; }
    if (L == 0) return codec_error(FEC_ERR_SHARD_NO_DATA);
    int present = 0;
    for (int i = 0; i < nsh; ++i) {
        if (shards[i].nil() || shards[i].len == 0) continue;
        if (shards[i].len != L) return codec_error(FEC_ERR_SHARD_SIZE);
        ++present;
    }
    if (present < k_) return codec_error(FEC_ERR_TOO_FEW_SHARDS);
    // the device decode takes uint32 present masks: n <= 32 (klauspost itself reconstructs up
    // to 256 shards; every code the reference builds has n <= 30, manager.go:54-90)
    if (nsh > FEC_MAX_DECODE_SHARDS) return codec_error(FEC_ERR_MAX_SHARD_NUM);
    uint32_t mask = 0;
    for (int i = 0; i < nsh; ++i)
        if (!shards[i].nil() && shards[i].len != 0) mask |= 1u << i;
    if (L > stride) return Error::text(fmt("shard len (%zu) exceeds the staging slot (%zu)", L, stride));
    for (int i = 0; i < nsh; ++i)
        if (mask >> i & 1u) {
            memcpy(dst + (size_t)i * stride, shards[i].data(), L);
            memset(dst + (size_t)i * stride + L, 0, std::min(stride, (L + 15) & ~(size_t)15) - L);
        }
    plan->len = L;
    plan->mask = mask;
    return Error::nil();
}

Error ReedSolomonScheme::stageRecoverPayloads(int biggest, const uint8_t* const* src, const size_t* slen,
                                              const uint8_t* const* rep, const size_t* rlen, uint8_t* dst,
                                              size_t stride, RecoverPlan* plan, const bool* skip) {
    // stageRecoverInput over the payloads themselves: the block is k sources (SSID order) and m
    // repairs (ParityID order); every check of reed_solomon.go:92-124 and ReconstructData, in order
    plan->nothing = false;
    plan->missing.clear();
    int nsrc = 0, nrep = 0;
    for (int i = 0; i < k_; ++i) nsrc += src[i] != nullptr;
    for (int p = 0; p < m_; ++p) nrep += rep[p] != nullptr;
    if (nsrc + nrep < k_) return Error::text(kNotRecoverable);   // isRecoverable (block.go:88)
    if (nsrc == k_) {
        plan->nothing = true;   // isComplete: nil, nil
        return Error::nil();
    }
    // addLengthToSourceSymbolPayload per present source (reed_solomon.go:70-89): a received
    // source payload has the capacity of a packet buffer
    const int shardLen = (int)kRepairPayloadMetadataLen + biggest;
    for (int i = 0; i < k_; ++i) {
        if (!src[i]) {
            plan->missing.push_back(i);
            continue;
        }
        if (shardLen > (int)kMaxPacketBufferSize)
            return Error::text(fmt("shard len (%d) is greater than capacity of payload (%d)", shardLen,
                                   (int)kMaxPacketBufferSize));
        if (shardLen < (int)kRepairPayloadMetadataLen) return Error::text(fmt("shard len (%d) is negative", biggest));
    }
    // enc.ReconstructData: shard length = the first non-empty shard's; all non-empty ones equal
    const int nsh = k_ + m_;
    auto len_of = [&](int i) -> size_t {
        return i < k_ ? (src[i] ? (size_t)shardLen : 0) : (rep[i - k_] ? rlen[i - k_] : 0);
    };
    size_t L = 0;
    for (int i = 0; i < nsh && !L; ++i) L = len_of(i);
    if (L == 0) return codec_error(FEC_ERR_SHARD_NO_DATA);
    int present = 0;
    uint32_t mask = 0;
    for (int i = 0; i < nsh; ++i) {
        const size_t li = len_of(i);
        if (li == 0) continue;
        if (li != L) return codec_error(FEC_ERR_SHARD_SIZE);
        ++present;
    }
    if (present < k_) return codec_error(FEC_ERR_TOO_FEW_SHARDS);
    if (nsh > FEC_MAX_DECODE_SHARDS) return codec_error(FEC_ERR_MAX_SHARD_NUM);
    if (L > stride) return Error::text(fmt("shard len (%zu) exceeds the staging slot (%zu)", L, stride));
    const size_t pad = std::min(stride, (L + 15) & ~(size_t)15) - L;
    for (int i = 0; i < nsh; ++i) {
        if (len_of(i) == 0) continue;
        mask |= 1u << i;
        if (skip && skip[i]) continue;
        uint8_t* d = dst + (size_t)i * stride;
        if (i < k_) {   // payload[:shardLen] of a zeroed packet buffer, BE16 length at [biggest]
            const size_t c = std::min(slen[i], L);
            if (c) memcpy(d, src[i], c);
            memset(d + c, 0, L - c);
            d[biggest] = (uint8_t)((uint16_t)slen[i] >> 8);
            d[biggest + 1] = (uint8_t)(slen[i] & 0xFF);
        } else {
            memcpy(d, rep[i - k_], L);
        }
        memset(d + L, 0, pad);
    }
    plan->len = L;
    plan->mask = mask;
    return Error::nil();
}

Error ReedSolomonScheme::finishRecover(const Block& b, const RecoverPlan& plan, const uint8_t* const* rebuilt,
                                       Slice* out) {
    // reed_solomon.go:126-135: concatenation of the rebuilt payloads, each cut to its trailer
    const size_t L = plan.len;
    const int big = b.biggestSourceSymbolLenSoFar;
    std::vector<uint8_t> acc;
    for (size_t r = 0; r < plan.missing.size(); ++r) {
        const uint8_t* sh = rebuilt[r];
        if (big < 0 || (size_t)big + 2 > L)   // Go: index out of range panic
            return Error::text(fmt("length trailer at %d outside shard of %zu bytes", big, L));
        const size_t payloadLen = ((size_t)sh[big] << 8) | sh[big + 1];
        if (payloadLen > L)   // Go: slice bounds out of range panic
            return Error::text(fmt("recovered payload length %zu exceeds shard length %zu", payloadLen, L));
        acc.insert(acc.end(), sh, sh + payloadLen);
    }
    *out = Slice::from(acc.data(), acc.size(), std::max(acc.size(), plan.missing.size() * (size_t)std::max(big, 0)));
    return Error::nil();
}

Error ReedSolomonScheme::recoverSymbolPayloads(Block& b, Slice* out) {   // reed_solomon.go:92-136
    *out = Slice{};
    const int nsh = std::max(0, b.totNumSourceSymbols + b.totNumRepairSymbols);
    size_t stride = 0;
    for (auto& kv : b.pidToRepairPayload) stride = std::max(stride, kv.second.len);
    stride = std::max<size_t>(1, std::max(stride, kRepairPayloadMetadataLen + (size_t)std::max(0, b.biggestSourceSymbolLenSoFar)));
    std::vector<uint8_t> host((size_t)nsh * stride + 1, 0);
    RecoverPlan plan;
    Error e = stageRecoverInput(b, host.data(), stride, &plan);
    if (!e.ok() || plan.nothing) return e;
    const size_t L = plan.len;
    // repack to the shard length (stride may exceed L)
    std::vector<uint8_t> dense((size_t)nsh * L, 0);
    for (int i = 0; i < nsh; ++i) memcpy(&dense[(size_t)i * L], &host[(size_t)i * stride], L);
    fec_ctx* ctx = nullptr;
    e = engine_->ctx(&ctx);
    if (!e.ok()) return e;
    uint32_t mask = plan.mask;
    int32_t st = 0;
    const int rc = fec_rs_reconstruct_batch(ctx, k_, m_, L, 1, dense.data(), (size_t)nsh * L, dense.data() + (size_t)k_ * L,
                                            (size_t)nsh * L, L, &mask, &st, FEC_HOST);
    if (rc) return codec_error(rc);
    std::vector<const uint8_t*> rebuilt;
    for (int i : plan.missing) rebuilt.push_back(&dense[(size_t)i * L]);
    return finishRecover(b, plan, rebuilt.data(), out);
}

// ------------------------------------------------------------------ XOR (xor.go)

// One source payload as the XOR scheme folds it in (xor.go:44-56): payload bytes at
// [0, len), big-endian uint16(len) XORed at [biggest, biggest+2), in an L-byte shard.
static bool xor_frame(const uint8_t* p, size_t len, int biggest, size_t L, uint8_t* dst) {
    if (biggest < 0 || (size_t)biggest + 2 > L || len > L) return false;
    memset(dst, 0, L);
    if (len) memcpy(dst, p, len);
    const uint16_t ln = (uint16_t)len;
    dst[biggest] ^= (uint8_t)(ln >> 8);
    dst[biggest + 1] ^= (uint8_t)(ln & 0xFF);
    return true;
}
static bool xor_frame(const Slice& p, int biggest, size_t L, uint8_t* dst) {
    return xor_frame(p.data(), p.len, biggest, L, dst);
}

static Error xor_reduce(std::shared_ptr<Engine>& engine, std::vector<uint8_t>& shards, int count, size_t L,
                        uint8_t* out) {
    if (count == 0) {
        memset(out, 0, L);
        return Error::nil();
    }
    fec_ctx* ctx = nullptr;
    Error e = engine->ctx(&ctx);
    if (!e.ok()) return e;
    const int rc = fec_xor_encode_batch(ctx, count, L, 1, shards.data(), (size_t)count * L, out, L, L, FEC_HOST);
    return rc ? codec_error(rc) : Error::nil();
}

Error XorScheme::stageRepairInput(Block& b, uint8_t* dst, size_t stride, size_t* shard_len, int* count) {
    // xor.go:14-33: the same checks in the same order, then every source framed into a slot
    if (!b.isComplete()) return Error::text(kIncomplete);
    if (b.totNumRepairSymbols != 1)
        return Error::text(fmt("xor only supports 1 repair symbol. Expected 1, received %d", b.totNumRepairSymbols));
    if (b.biggestSourceSymbolLenSoFar > (int)kMaxFECPacketBufferSize) return too_big(b.biggestSourceSymbolLenSoFar);
    if (b.biggestSourceSymbolLenSoFar < 0) return Error::text("negative repair payload length");
    const size_t L = kRepairPayloadMetadataLen + (size_t)b.biggestSourceSymbolLenSoFar;
    if (L > stride) return Error::text(fmt("shard len (%zu) exceeds the staging slot (%zu)", L, stride));
    int i = 0;
    for (auto& kv : b.ssidToSourcePayload) {
        uint8_t* slot = dst + (size_t)i * stride;
        if (!xor_frame(kv.second, b.biggestSourceSymbolLenSoFar, L, slot))
            return Error::text(fmt("source payload of %zu bytes overruns the %zu-byte repair symbol",
                                   kv.second.len, L));   // Go: index out of range panic
        memset(slot + L, 0, std::min(stride, (L + 15) & ~(size_t)15) - L);
        ++i;
    }
    *shard_len = L;
    *count = i;
    return Error::nil();
}

Error XorScheme::repairSymbols(Block& b, std::vector<RepairFrame>* out) {   // xor.go:14-42
    out->clear();
    const size_t stride = kRepairPayloadMetadataLen + (size_t)std::max(0, b.biggestSourceSymbolLenSoFar);
    std::vector<uint8_t> shards(b.ssidToSourcePayload.size() * stride + 1);
    size_t L = 0;
    int count = 0;
    Error e = stageRepairInput(b, shards.data(), stride, &L, &count);
    if (!e.ok()) return e;
    Slice rep = Slice::make(L, L);
    e = xor_reduce(engine_, shards, count, L, rep.data());
    if (!e.ok()) return e;
    out->resize(1);
    (*out)[0].block_id = b.id;
    (*out)[0].parity_id = 0;
    (*out)[0].payload = rep;
    return Error::nil();
}

Error XorScheme::stageRecoverInput(Block& b, uint8_t* dst, size_t stride, size_t slots, bool* nothing, int* count) {
    // xor.go:66-86 up to the XOR loop: the same checks, then the repair payloads (whole) and
    // the present sources (framed) into dst + i*stride; slots past the inputs are zeroed
    *nothing = false;
    if (!b.isRecoverable()) return Error::text(kNotRecoverable);
    if (b.isComplete()) {
        *nothing = true;
        return Error::nil();
    }
    const size_t L = std::min(stride, kMaxPacketBufferSize);
    const size_t n = b.pidToRepairPayload.size() + b.ssidToSourcePayload.size();
    if (n > slots) return Error::text(fmt("%zu XOR inputs exceed the %zu staging slots", n, slots));
    int i = 0;
    for (auto& kv : b.pidToRepairPayload) {   // xorRepair: whole repair payload
        if (kv.second.len > L) return Error::text("repair payload longer than the packet buffer");
        uint8_t* slot = dst + (size_t)i * stride;
        memset(slot, 0, stride);
        if (kv.second.len) memcpy(slot, kv.second.data(), kv.second.len);
        ++i;
    }
    for (auto& kv : b.ssidToSourcePayload) {
        uint8_t* slot = dst + (size_t)(i++) * stride;
        memset(slot, 0, stride);
        if (!xor_frame(kv.second, b.biggestSourceSymbolLenSoFar, L, slot))
            return Error::text("source payload overruns the packet buffer");
    }
    for (size_t z = (size_t)i; z < slots; ++z) memset(dst + z * stride, 0, stride);
    *count = i;
    return Error::nil();
}

Error XorScheme::stageRecoverPayloads(int k, int m, int biggest, const uint8_t* const* src, const size_t* slen,
                                     const uint8_t* const* rep, const size_t* rlen, uint8_t* dst, size_t stride,
                                     size_t slots, bool* nothing, int* count) {
    // stageRecoverInput over the payloads: repairs (ParityID order) whole, then the present
    // sources (SSID order) framed, as xor.go:78-84 walks the block's maps
    *nothing = false;
    int nsrc = 0, nrep = 0;
    for (int i = 0; i < k; ++i) nsrc += src[i] != nullptr;
    for (int p = 0; p < m; ++p) nrep += rep[p] != nullptr;
    if (nsrc + nrep < k) return Error::text(kNotRecoverable);
    if (nsrc == k) {
        *nothing = true;
        return Error::nil();
    }
    const size_t L = std::min(stride, kMaxPacketBufferSize);
    const size_t n = (size_t)(nrep + nsrc);
    if (n > slots) return Error::text(fmt("%zu XOR inputs exceed the %zu staging slots", n, slots));
    int i = 0;
    for (int p = 0; p < m; ++p) {
        if (!rep[p]) continue;
        if (rlen[p] > L) return Error::text("repair payload longer than the packet buffer");
        uint8_t* slot = dst + (size_t)(i++) * stride;
        memset(slot, 0, stride);
        if (rlen[p]) memcpy(slot, rep[p], rlen[p]);
    }
    for (int j = 0; j < k; ++j) {
        if (!src[j]) continue;
        uint8_t* slot = dst + (size_t)(i++) * stride;
        memset(slot, 0, stride);
        if (!xor_frame(src[j], slen[j], biggest, L, slot)) return Error::text("source payload overruns the packet buffer");
    }
    for (size_t z = (size_t)i; z < slots; ++z) memset(dst + z * stride, 0, stride);
    *count = i;
    return Error::nil();
}

Error XorScheme::finishRecover(Block& b, const uint8_t* rec, size_t len, Slice* out) {
    // xor.go:86-103: the length trailer names the payload; it is stored for the missing SSID
    Slice full = Slice::make(kMaxPacketBufferSize, kMaxPacketBufferSize);
    memcpy(full.data(), rec, std::min(len, kMaxPacketBufferSize));
    const int big = b.biggestSourceSymbolLenSoFar;
    if (big < 0 || (size_t)big + 2 > kMaxPacketBufferSize) return Error::text("length trailer outside the packet buffer");
    const size_t payloadLen = ((size_t)full.data()[big] << 8) | full.data()[big + 1];
    if (payloadLen > kMaxPacketBufferSize) return Error::text("recovered payload length exceeds the packet buffer");
    Slice recovered = full.reslice(0, payloadLen);
    for (SourceSymbolID ssid = b.smallestSSID;; ++ssid) {
        if (!b.ssidToSourcePayload.count(ssid)) b.ssidToSourcePayload[ssid] = recovered;
        if (ssid == b.largestSSID) break;
    }
    if (!b.isComplete()) return Error::text("block is not complete after recovery");
    *out = recovered;
    return Error::nil();
}

Error XorScheme::recoverSymbolPayloads(Block& b, Slice* out) {   // xor.go:66-104
    *out = Slice{};
    const size_t L = kMaxPacketBufferSize;
    const size_t slots = b.pidToRepairPayload.size() + b.ssidToSourcePayload.size();
    std::vector<uint8_t> shards(std::max<size_t>(slots, 1) * L, 0);
    bool nothing = false;
    int count = 0;
    Error e = stageRecoverInput(b, shards.data(), L, slots, &nothing, &count);
    if (!e.ok() || nothing) return e;
    std::vector<uint8_t> rec(L, 0);
    e = xor_reduce(engine_, shards, count, L, rec.data());
    if (!e.ok()) return e;
    return finishRecover(b, rec.data(), L, out);
}

// ------------------------------------------------------------------ manager (manager.go)

Error Manager::New(std::unique_ptr<BlockFECScheme> scheme, int k, int m, std::unique_ptr<Manager>* out) {
    // manager.go:96-109
    if (k < 0 || m < 0)
        return Error::text(fmt("numTotSourceSymbols (%d) and numTotRepairSymbols (%d) may not be negative", k, m));
    std::unique_ptr<Manager> mg(new Manager());
    mg->scheme_ = std::move(scheme);
    mg->numTotSourceSymbols_ = k;
    mg->numTotRepairSymbols_ = m;
    *out = std::move(mg);
    return Error::nil();
}

SourceSymbolID Manager::NextSSID() {   // manager.go:111-117
    std::lock_guard<std::mutex> g(nextSIDMutex_);
    return nextSID_++;
}

BlockID Manager::sidToBlockID(SourceSymbolID sid) const {   // manager.go:119-121
    return numTotSourceSymbols_ > 0 ? sid / (uint64_t)numTotSourceSymbols_ : 0;   // Go: divide-by-zero panic
}

Manager::BlockStatus& Manager::statusFor(BlockID id) {
    auto it = blockStatuses_.find(id);
    if (it == blockStatuses_.end()) {
        BlockStatus st;
        st.block.reset(new Block(Block::New(id, numTotSourceSymbols_, numTotRepairSymbols_)));
        it = blockStatuses_.emplace(id, std::move(st)).first;
    }
    return it->second;
}

Error Manager::AddSourceSymbolFrame(const SourceSymbolFrame& f, std::vector<RepairFrame>* out) {   // :123-158
    out->clear();
    BlockStatus& bs = statusFor(sidToBlockID(f.ssid));
    if (bs.isProcessed) return Error::nil();
    Error e = bs.block->addSourceSymbol(f);
    if (!e.ok()) return e;
    if (bs.block->isComplete()) {
        std::vector<RepairFrame> rep;
        e = scheme_->repairSymbols(*bs.block, &rep);
        if (!e.ok()) return e;
        bs.block.reset();
        bs.isProcessed = true;
        *out = std::move(rep);
    }
    return Error::nil();
}

Error Manager::AddSourceSymbolFrameBatched(const SourceSymbolFrame& f, BatchEncoder* enc, RepairQueue* q) {
    // manager.go:123-158 with repairSymbols replaced by staging into the batch encoder
    if (!enc) return Error::text("nil batch encoder");
    BlockStatus& bs = statusFor(sidToBlockID(f.ssid));
    if (bs.isProcessed) return Error::nil();
    Error e = bs.block->addSourceSymbol(f);
    if (!e.ok()) return e;
    if (bs.block->isComplete()) {
        e = enc->Submit(*bs.block, q);
        if (!e.ok()) return e;
        bs.block.reset();
        bs.isProcessed = true;
    }
    return Error::nil();
}

Error Manager::HandleRepairFrameBatched(const RepairFrame& f, BatchDecoder* dec, RecoveredQueue* q) {
    // manager.go:160-198 with recoverSymbolPayloads replaced by staging into the batch decoder
    if (!dec) return Error::text("nil batch decoder");
    BlockStatus& bs = statusFor(f.block_id);
    if (bs.isProcessed) return Error::nil();
    Error e = bs.block->addRepairSymbol(f);
    if (!e.ok()) return e;
    if (bs.block->isRecoverable()) {
        e = dec->Submit(*bs.block, q);
        if (!e.ok()) return e;
        bs.block.reset();
        bs.isProcessed = true;
    }
    return Error::nil();
}

Error Manager::HandleRepairFrame(const RepairFrame& f, Slice* out) {   // manager.go:160-198
    *out = Slice{};
    BlockStatus& bs = statusFor(f.block_id);
    if (bs.isProcessed) return Error::nil();
    Error e = bs.block->addRepairSymbol(f);
    if (!e.ok()) return e;
    if (bs.block->isRecoverable()) {
        Slice rec;
        e = scheme_->recoverSymbolPayloads(*bs.block, &rec);
        if (!e.ok()) return e;
        bs.block.reset();
        bs.isProcessed = true;
        *out = rec;
    }
    return Error::nil();
}

Error Manager::HandleSourceSymbolFrame(const SourceSymbolFrame& f, Slice* out, Slice* recovered) {
    // manager.go:200-227 (+ the optional recover-on-source trigger, default off)
    *out = Slice{};
    if (recovered) *recovered = Slice{};
    BlockStatus& bs = statusFor(sidToBlockID(f.ssid));
    if (bs.isProcessed) return Error::nil();
    Error e = bs.block->addSourceSymbol(f);
    if (!e.ok()) return e;
    if (bs.block->isComplete()) {
        bs.block.reset();
        bs.isProcessed = true;
    } else if (recoverOnSource_ && bs.block->isRecoverable()) {
        Slice rec;
        e = scheme_->recoverSymbolPayloads(*bs.block, &rec);
        if (!e.ok()) return e;
        bs.block.reset();
        bs.isProcessed = true;
        if (recovered) *recovered = rec;
    }
    *out = f.payload;
    return Error::nil();
}

Error Manager::HandleSourceSymbolFrameBatched(const SourceSymbolFrame& f, Slice* out, BatchDecoder* dec,
                                              RecoveredQueue* q) {
    *out = Slice{};
    if (!dec) return Error::text("nil batch decoder");
    BlockStatus& bs = statusFor(sidToBlockID(f.ssid));
    if (bs.isProcessed) return Error::nil();
    Error e = bs.block->addSourceSymbol(f);
    if (!e.ok()) return e;
    if (bs.block->isComplete()) {
        bs.block.reset();
        bs.isProcessed = true;
    } else if (recoverOnSource_ && bs.block->isRecoverable()) {
        e = dec->Submit(*bs.block, q);
        if (!e.ok()) return e;
        bs.block.reset();
        bs.isProcessed = true;
    }
    *out = f.payload;
    return Error::nil();
}

static Error new_manager(DecoderFECScheme id, std::shared_ptr<Engine> engine, std::unique_ptr<Manager>* out) {
    // manager.go:50-94 (NewSender and NewReceiver are identical)
    out->reset();
    switch (id) {
        case FECDisabled:
            return Error::nil();
        case XORFECScheme:
            return Manager::New(std::unique_ptr<BlockFECScheme>(new XorScheme(std::move(engine))), 2, 1, out);
        case ReedSolomonFECScheme: {
            std::unique_ptr<ReedSolomonScheme> rs;
            Error e = ReedSolomonScheme::New(20, 10, std::move(engine), &rs);
            if (!e.ok()) return e;
            return Manager::New(std::move(rs), 20, 10, out);
        }
        default:
            return Error::text(fmt("unknown FEC scheme: %d", (int)id));
    }
}

Error NewSender(DecoderFECScheme id, std::shared_ptr<Engine> engine, std::unique_ptr<Manager>* out) {
    return new_manager(id, std::move(engine), out);
}

Error NewReceiver(DecoderFECScheme id, std::shared_ptr<Engine> engine, std::unique_ptr<Manager>* out) {
    return new_manager(id, std::move(engine), out);
}

}  // namespace fec

// ------------------------------------------------------------------ C ABI (include/fec_scheme.h)

struct fec_block {
    fec::Block b;
};
struct fec_scheme {
    std::unique_ptr<fec::BlockFECScheme> s;
};
struct fec_manager {
    std::unique_ptr<fec::Manager> m;
};
struct fec_frames {
    std::vector<fec::RepairFrame> f;
};
struct fec_bytes {
    fec::Slice s;
};

static thread_local std::string t_last_error;

namespace fec {
namespace cabi {
// Shared by the C ABIs of this library (fec_scheme.h, fec_batch.h, fec_go.h): a nil error is 0;
// otherwise the Go text goes to fec_last_error() and the code (FEC_ERR_SCHEME for Go-level
// errors) is returned.
int report(const fec::Error& e) {
    if (e.ok()) {
        t_last_error.clear();
        return FEC_OK;
    }
    t_last_error = e.msg;
    return e.code ? e.code : FEC_ERR_SCHEME;
}

std::shared_ptr<fec::Engine> engine_for(int device) {
    // one engine (one fec_ctx, created lazily) per device per thread
    static thread_local std::map<int, std::shared_ptr<fec::Engine>> engines;
    auto& e = engines[device];
    if (!e) e = std::make_shared<fec::Engine>(device);
    return e;
}
}  // namespace cabi
}  // namespace fec

using fec::cabi::engine_for;
using fec::cabi::report;

extern "C" {

const char* fec_last_error(void) { return t_last_error.c_str(); }

fec_block* fec_block_new(uint64_t id, int tot_src, int tot_rep) {
    fec_block* b = new fec_block();
    b->b = fec::Block::New(id, tot_src, tot_rep);
    return b;
}

fec_block* fec_block_literal(uint64_t id, int tot_src, int tot_rep, int biggest, uint64_t smallest, uint64_t largest) {
    fec_block* b = new fec_block();
    b->b.id = id;
    b->b.totNumSourceSymbols = tot_src;
    b->b.totNumRepairSymbols = tot_rep;
    b->b.biggestSourceSymbolLenSoFar = biggest;
    b->b.smallestSSID = smallest;
    b->b.largestSSID = largest;
    return b;
}

void fec_block_free(fec_block* b) { delete b; }

int fec_block_put_source(fec_block* b, uint64_t ssid, const uint8_t* p, size_t len, size_t cap) {
    if (!b || (len && !p)) return FEC_ERR_INVALID_ARG;
    b->b.ssidToSourcePayload[ssid] = fec::Slice::from(p, len, cap);
    return FEC_OK;
}

int fec_block_put_repair(fec_block* b, uint64_t pid, const uint8_t* p, size_t len) {
    if (!b || (len && !p)) return FEC_ERR_INVALID_ARG;
    b->b.pidToRepairPayload[pid] = fec::Slice::from(p, len, len);
    return FEC_OK;
}

int fec_block_add_source_symbol(fec_block* b, uint64_t ssid, const uint8_t* p, size_t len, size_t cap) {
    if (!b || (len && !p)) return FEC_ERR_INVALID_ARG;
    fec::SourceSymbolFrame f{ssid, fec::Slice::from(p, len, cap)};
    return report(b->b.addSourceSymbol(f));
}

int fec_block_add_repair_symbol(fec_block* b, uint64_t block_id, uint64_t pid, const uint8_t* p, size_t len) {
    if (!b || (len && !p)) return FEC_ERR_INVALID_ARG;
    fec::RepairFrame f{block_id, pid, fec::Slice::from(p, len, len)};
    return report(b->b.addRepairSymbol(f));
}

int fec_block_is_recoverable(const fec_block* b) { return b && b->b.isRecoverable(); }
int fec_block_is_complete(const fec_block* b) { return b && b->b.isComplete(); }
int fec_block_biggest(const fec_block* b) { return b ? b->b.biggestSourceSymbolLenSoFar : 0; }
int fec_block_num_sources(const fec_block* b) { return b ? (int)b->b.ssidToSourcePayload.size() : 0; }

long fec_block_get_source(const fec_block* b, uint64_t ssid, uint8_t* out, size_t out_cap) {
    if (!b) return -1;
    auto it = b->b.ssidToSourcePayload.find(ssid);
    if (it == b->b.ssidToSourcePayload.end()) return -1;
    const size_t n = std::min(out_cap, it->second.len);
    if (n && out) memcpy(out, it->second.data(), n);
    return (long)it->second.len;
}

fec_scheme* fec_scheme_new(int scheme_id, int k, int m, int device) {
    fec_scheme* s = new fec_scheme();
    if (scheme_id == fec::XORFECScheme) {
        s->s.reset(new fec::XorScheme(engine_for(device)));
    } else if (scheme_id == fec::ReedSolomonFECScheme) {
        std::unique_ptr<fec::ReedSolomonScheme> rs;
        if (report(fec::ReedSolomonScheme::New(k, m, engine_for(device), &rs)) != FEC_OK) {
            delete s;
            return nullptr;
        }
        s->s = std::move(rs);
    } else {
        report(fec::Error::text(fec::fmt("unknown FEC scheme: %d", scheme_id)));
        delete s;
        return nullptr;
    }
    t_last_error.clear();
    return s;
}

void fec_scheme_free(fec_scheme* s) { delete s; }

int fec_scheme_repair_symbols(fec_scheme* s, fec_block* b, fec_frames** out) {
    if (!s || !b || !out) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    std::vector<fec::RepairFrame> f;
    const int rc = report(s->s->repairSymbols(b->b, &f));
    if (rc == FEC_OK) *out = new fec_frames{std::move(f)};
    return rc;
}

int fec_scheme_recover_symbol_payloads(fec_scheme* s, fec_block* b, fec_bytes** out) {
    if (!s || !b || !out) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    fec::Slice r;
    const int rc = report(s->s->recoverSymbolPayloads(b->b, &r));
    if (rc == FEC_OK && !r.nil()) *out = new fec_bytes{r};
    return rc;
}

size_t fec_frames_count(const fec_frames* f) { return f ? f->f.size() : 0; }

int fec_frames_get(const fec_frames* f, size_t i, uint64_t* block_id, uint64_t* parity_id, const uint8_t** payload,
                   size_t* len) {
    if (!f || i >= f->f.size()) return FEC_ERR_INVALID_ARG;
    const fec::RepairFrame& r = f->f[i];
    if (block_id) *block_id = r.block_id;
    if (parity_id) *parity_id = r.parity_id;
    if (payload) *payload = r.payload.data();
    if (len) *len = r.payload.len;
    return FEC_OK;
}

void fec_frames_free(fec_frames* f) { delete f; }

const uint8_t* fec_bytes_data(const fec_bytes* b) { return b ? b->s.data() : nullptr; }
size_t fec_bytes_len(const fec_bytes* b) { return b ? b->s.len : 0; }
void fec_bytes_free(fec_bytes* b) { delete b; }

static fec_manager* make_manager(fec::Error (*fn)(fec::DecoderFECScheme, std::shared_ptr<fec::Engine>,
                                                  std::unique_ptr<fec::Manager>*),
                                 int scheme_id, int device, int* err) {
    std::unique_ptr<fec::Manager> m;
    const int rc = report(fn((fec::DecoderFECScheme)scheme_id, engine_for(device), &m));
    if (err) *err = rc;
    if (rc != FEC_OK || !m) return nullptr;
    return new fec_manager{std::move(m)};
}

fec_manager* fec_manager_new_sender(int scheme_id, int device, int* err) {
    return make_manager(fec::NewSender, scheme_id, device, err);
}

fec_manager* fec_manager_new_receiver(int scheme_id, int device, int* err) {
    return make_manager(fec::NewReceiver, scheme_id, device, err);
}

fec_manager* fec_manager_new(int scheme_id, int k, int m, int device, int* err) {
    std::unique_ptr<fec::BlockFECScheme> s;
    fec::Error e;
    if (scheme_id == fec::XORFECScheme) {
        s.reset(new fec::XorScheme(engine_for(device)));
    } else if (scheme_id == fec::ReedSolomonFECScheme) {
        std::unique_ptr<fec::ReedSolomonScheme> rs;
        e = fec::ReedSolomonScheme::New(k, m, engine_for(device), &rs);
        s = std::move(rs);
    } else {
        e = fec::Error::text(fec::fmt("unknown FEC scheme: %d", scheme_id));
    }
    std::unique_ptr<fec::Manager> mg;
    if (e.ok()) e = fec::Manager::New(std::move(s), k, m, &mg);
    const int rc = report(e);
    if (err) *err = rc;
    return rc == FEC_OK ? new fec_manager{std::move(mg)} : nullptr;
}

void fec_manager_free(fec_manager* m) { delete m; }

uint64_t fec_manager_next_ssid(fec_manager* m) { return m ? m->m->NextSSID() : 0; }

uint64_t fec_manager_block_id(const fec_manager* m, uint64_t ssid) { return m ? m->m->sidToBlockID(ssid) : 0; }

int fec_manager_add_source_symbol_frame(fec_manager* m, uint64_t ssid, const uint8_t* p, size_t len, size_t cap,
                                        fec_frames** out) {
    if (!m || !out || (len && !p)) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    std::vector<fec::RepairFrame> f;
    const int rc = report(m->m->AddSourceSymbolFrame(fec::SourceSymbolFrame{ssid, fec::Slice::from(p, len, cap)}, &f));
    if (rc == FEC_OK && !f.empty()) *out = new fec_frames{std::move(f)};
    return rc;
}

int fec_manager_handle_repair_frame(fec_manager* m, uint64_t block_id, uint64_t pid, const uint8_t* p, size_t len,
                                    fec_bytes** out) {
    if (!m || !out || (len && !p)) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    fec::Slice r;
    const int rc = report(m->m->HandleRepairFrame(fec::RepairFrame{block_id, pid, fec::Slice::from(p, len, len)}, &r));
    if (rc == FEC_OK && !r.nil()) *out = new fec_bytes{r};
    return rc;
}

int fec_manager_handle_source_symbol_frame(fec_manager* m, uint64_t ssid, const uint8_t* p, size_t len, size_t cap,
                                           fec_bytes** out) {
    if (!m || !out || (len && !p)) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    fec::Slice r;
    const int rc =
        report(m->m->HandleSourceSymbolFrame(fec::SourceSymbolFrame{ssid, fec::Slice::from(p, len, cap)}, &r));
    if (rc == FEC_OK && !r.nil()) *out = new fec_bytes{r};
    return rc;
}

int fec_manager_set_recover_on_source(fec_manager* m, int on) {
    if (!m) return FEC_ERR_INVALID_ARG;
    m->m->SetRecoverOnSource(on != 0);
    return FEC_OK;
}

int fec_manager_handle_source_symbol_frame_recover(fec_manager* m, uint64_t ssid, const uint8_t* p, size_t len,
                                                   size_t cap, fec_bytes** out, fec_bytes** recovered) {
    if (!m || !out || !recovered || (len && !p)) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    *recovered = nullptr;
    fec::Slice r, rec;
    const int rc =
        report(m->m->HandleSourceSymbolFrame(fec::SourceSymbolFrame{ssid, fec::Slice::from(p, len, cap)}, &r, &rec));
    if (rc == FEC_OK && !r.nil()) *out = new fec_bytes{r};
    if (rc == FEC_OK && !rec.nil()) *recovered = new fec_bytes{rec};
    return rc;
}

}  // extern "C"

// ------------------------------------------------------------------ C ABI (include/fec_batch.h)

struct fec_repair_queue {
    std::unique_ptr<fec::RepairQueue> q;
    std::atomic<uint64_t> has_data{0};
};
struct fec_batch_encoder {
    std::unique_ptr<fec::BatchEncoder> e;
};

extern "C" {

fec_repair_queue* fec_repair_queue_new(size_t max_len) {
    fec_repair_queue* r = new fec_repair_queue();
    r->q.reset(new fec::RepairQueue([r] { r->has_data.fetch_add(1); },
                                    max_len ? max_len : fec::RepairQueue::kMaxRepairSendQueueLen));
    return r;
}

void fec_repair_queue_free(fec_repair_queue* q) { delete q; }

int fec_repair_queue_add(fec_repair_queue* q, uint64_t block_id, uint64_t parity_id, const uint8_t* p, size_t len) {
    if (!q || (len && !p)) return FEC_ERR_INVALID_ARG;
    return report(q->q->Add(fec::RepairFrame{block_id, parity_id, fec::Slice::from(p, len, len)}));
}

int fec_repair_queue_peek(fec_repair_queue* q, uint64_t* block_id, uint64_t* parity_id, const uint8_t** payload,
                          size_t* len, size_t* cap) {
    if (!q) return FEC_ERR_INVALID_ARG;
    const fec::RepairFrame* f = q->q->Peek();
    if (!f) return 0;
    if (block_id) *block_id = f->block_id;
    if (parity_id) *parity_id = f->parity_id;
    if (payload) *payload = f->payload.data();
    if (len) *len = f->payload.len;
    if (cap) *cap = f->payload.cap;
    return 1;
}

void fec_repair_queue_pop(fec_repair_queue* q) {
    if (q) q->q->Pop();
}

size_t fec_repair_queue_len(fec_repair_queue* q) { return q ? q->q->Len() : 0; }

uint64_t fec_repair_queue_has_data_calls(fec_repair_queue* q) { return q ? q->has_data.load() : 0; }

void fec_repair_queue_close(fec_repair_queue* q, const char* msg) {
    if (q) q->q->CloseWithError(fec::Error::text(msg && *msg ? msg : "closed"));
}

fec_batch_encoder* fec_batch_encoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int* err) {
    std::unique_ptr<fec::BatchEncoder> e;
    const int rc = report(fec::BatchEncoder::New((fec::DecoderFECScheme)scheme_id, k, m, max_blocks,
                                                 engine_for(device), &e));
    if (err) *err = rc;
    if (rc) return nullptr;
    return new fec_batch_encoder{std::move(e)};
}

void fec_batch_encoder_free(fec_batch_encoder* e) { delete e; }

int fec_batch_encoder_submit(fec_batch_encoder* e, fec_block* b, fec_repair_queue* q) {
    if (!e || !b || !q) return FEC_ERR_INVALID_ARG;
    return report(e->e->Submit(b->b, q->q.get()));
}

int fec_batch_encoder_flush(fec_batch_encoder* e) { return e ? report(e->e->Flush()) : FEC_ERR_INVALID_ARG; }

int fec_batch_encoder_poll(fec_batch_encoder* e, size_t* blocks) {
    return e ? report(e->e->Poll(blocks)) : FEC_ERR_INVALID_ARG;
}

int fec_batch_encoder_drain(fec_batch_encoder* e, size_t* blocks) {
    return e ? report(e->e->Drain(blocks)) : FEC_ERR_INVALID_ARG;
}

size_t fec_batch_encoder_staged(const fec_batch_encoder* e) { return e ? e->e->Staged() : 0; }

size_t fec_batch_encoder_in_flight(const fec_batch_encoder* e) { return e ? e->e->InFlight() : 0; }
size_t fec_batch_encoder_backlog(const fec_batch_encoder* e) { return e ? e->e->Backlog() : 0; }

int fec_manager_add_source_symbol_frame_batched(fec_manager* m, uint64_t ssid, const uint8_t* p, size_t len,
                                                size_t cap, fec_batch_encoder* e, fec_repair_queue* q) {
    if (!m || !e || !q || (len && !p)) return FEC_ERR_INVALID_ARG;
    fec::SourceSymbolFrame f{ssid, fec::Slice::from(p, len, cap)};
    return report(m->m->AddSourceSymbolFrameBatched(f, e->e.get(), q->q.get()));
}


}  // extern "C"

struct fec_recovered_queue {
    fec::RecoveredQueue q;
};
struct fec_batch_decoder {
    std::unique_ptr<fec::BatchDecoder> d;
};

extern "C" {

fec_recovered_queue* fec_recovered_queue_new(void) { return new fec_recovered_queue(); }

void fec_recovered_queue_free(fec_recovered_queue* q) { delete q; }

size_t fec_recovered_queue_len(fec_recovered_queue* q) { return q ? q->q.Len() : 0; }

int fec_recovered_queue_pop(fec_recovered_queue* q, uint64_t* block_id, fec_bytes** out) {
    if (!q || !out) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    fec::RecoveredQueue::Item it;
    if (!q->q.Pop(&it)) return 0;
    if (block_id) *block_id = it.block_id;
    *out = new fec_bytes{it.payload};
    return 1;
}

fec_batch_decoder* fec_batch_decoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int* err) {
    std::unique_ptr<fec::BatchDecoder> d;
    const int rc = report(fec::BatchDecoder::New((fec::DecoderFECScheme)scheme_id, k, m, max_blocks,
                                                 engine_for(device), &d));
    if (err) *err = rc;
    if (rc) return nullptr;
    return new fec_batch_decoder{std::move(d)};
}

void fec_batch_decoder_free(fec_batch_decoder* d) { delete d; }

int fec_batch_decoder_submit(fec_batch_decoder* d, fec_block* b, fec_recovered_queue* q, int* staged) {
    if (!d || !b || !q) return FEC_ERR_INVALID_ARG;
    bool st = false;
    const int rc = report(d->d->Submit(b->b, &q->q, &st));
    if (staged) *staged = st ? 1 : 0;
    return rc;
}

int fec_batch_decoder_flush(fec_batch_decoder* d) { return d ? report(d->d->Flush()) : FEC_ERR_INVALID_ARG; }

int fec_batch_decoder_poll(fec_batch_decoder* d, size_t* blocks) {
    return d ? report(d->d->Poll(blocks)) : FEC_ERR_INVALID_ARG;
}

int fec_batch_decoder_drain(fec_batch_decoder* d, size_t* blocks) {
    return d ? report(d->d->Drain(blocks)) : FEC_ERR_INVALID_ARG;
}

size_t fec_batch_decoder_staged(const fec_batch_decoder* d) { return d ? d->d->Staged() : 0; }

size_t fec_batch_decoder_in_flight(const fec_batch_decoder* d) { return d ? d->d->InFlight() : 0; }

int fec_manager_handle_repair_frame_batched(fec_manager* m, uint64_t block_id, uint64_t parity_id, const uint8_t* p,
                                            size_t len, fec_batch_decoder* d, fec_recovered_queue* q) {
    if (!m || !d || !q || (len && !p)) return FEC_ERR_INVALID_ARG;
    fec::RepairFrame f{block_id, parity_id, fec::Slice::from(p, len, len)};
    return report(m->m->HandleRepairFrameBatched(f, d->d.get(), &q->q));
}

int fec_manager_handle_source_symbol_frame_batched(fec_manager* m, uint64_t ssid, const uint8_t* p, size_t len,
                                                   size_t cap, fec_bytes** out, fec_batch_decoder* d,
                                                   fec_recovered_queue* q) {
    if (!m || !out || !d || !q || (len && !p)) return FEC_ERR_INVALID_ARG;
    *out = nullptr;
    fec::Slice r;
    const int rc = report(m->m->HandleSourceSymbolFrameBatched(
        fec::SourceSymbolFrame{ssid, fec::Slice::from(p, len, cap)}, &r, d->d.get(), &q->q));
    if (rc == FEC_OK && !r.nil()) *out = new fec_bytes{r};
    return rc;
}

int fec_batch_encoder_submit_payloads(fec_batch_encoder* e, uint64_t block_id, const uint8_t* const* payloads,
                                      const size_t* lens, int count, fec_repair_queue* q) {
    if (!e || !q) return FEC_ERR_INVALID_ARG;
    return report(e->e->SubmitPayloads(block_id, payloads, lens, count, q->q.get()));
}

}  // extern "C"
