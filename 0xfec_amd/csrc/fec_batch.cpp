// fec_batch.cpp — RepairQueue (repair_queue.go restated) and BatchEncoder (deferred, batched
// repair-symbol generation on the GPU). Design and contracts: include/fec_batch.hpp.
#include "../../include/fec_batch.hpp"

#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/fec_hip.h"

namespace fec {

// ------------------------------------------------------------------ RepairQueue

Error RepairQueue::Add(RepairFrame f) {   // repair_queue.go:40-69
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (closed_) return closeErr_.ok() ? Error::text("repair queue closed") : closeErr_;
        // the reference panics("repair queue full") here (repair_queue.go:53)
        if (q_.size() >= maxLen_) return Error::text("repair queue full");
        q_.push_back(std::move(f));
    }
    if (hasData_) hasData_();
    return Error::nil();
}

const RepairFrame* RepairQueue::Peek() {   // repair_queue.go:73-80
    std::lock_guard<std::mutex> lk(mu_);
    return q_.empty() ? nullptr : &q_.front();
}

void RepairQueue::Pop() {   // repair_queue.go:82-90
    std::lock_guard<std::mutex> lk(mu_);
    if (!q_.empty()) q_.pop_front();
}

void RepairQueue::CloseWithError(Error e) {   // repair_queue.go:92-95
    std::lock_guard<std::mutex> lk(mu_);
    closeErr_ = std::move(e);
    closed_ = true;
}

size_t RepairQueue::Len() {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
}

bool RepairQueue::Closed() {
    std::lock_guard<std::mutex> lk(mu_);
    return closed_;
}

// ------------------------------------------------------------------ BatchEncoder

namespace {
constexpr size_t kSlotMax = (kMaxFECPacketBufferSize + kRepairPayloadMetadataLen + 15) & ~size_t(15);   // 1440
// Receive side: a repair payload may be as long as a packet buffer (XOR recovery accepts up to
// MaxPacketBufferSize, xor.go:76-86), so decoder slots hold 1452 bytes.
constexpr size_t kDecSlotMax = (kMaxPacketBufferSize + 15) & ~size_t(15);   // 1456
size_t round16(size_t x) { return (x + 15) & ~size_t(15); }
Error hip_error(hipError_t e, const char* what) {
    (void)hipGetLastError();
    return Error{std::string(what) + ": " + hipGetErrorString(e), FEC_ERR_HIP};
}
Error codec_rc(int rc) { return rc ? Error{fec_strerror(rc), rc} : Error::nil(); }
}  // namespace

Error BatchEncoder::New(DecoderFECScheme scheme, int k, int m, size_t maxBlocks, std::shared_ptr<Engine> engine,
                        std::unique_ptr<BatchEncoder>* out) {
    out->reset();
    if (maxBlocks == 0) return Error::text("batch must hold at least one block");
    std::unique_ptr<BatchEncoder> e(new BatchEncoder(scheme, k, m, maxBlocks, std::move(engine)));
    if (scheme == ReedSolomonFECScheme) {
        Error err = ReedSolomonScheme::New(k, m, e->engine_, &e->rs_);
        if (!err.ok()) return err;
    } else if (scheme == XORFECScheme) {
        if (m != 1) return Error::text("xor only supports 1 repair symbol");
        if (k < 1 || k > 255) return Error::text("invalid number of source symbols");
        e->xor_.reset(new XorScheme(e->engine_));
    } else {
        return Error::text("no FEC scheme");
    }
    *out = std::move(e);
    return Error::nil();
}

BatchEncoder::~BatchEncoder() {
    for (Set& s : sets_) {
        if (s.inFlight && s.done) (void)hipEventSynchronize((hipEvent_t)s.done);
        if (s.done) (void)hipEventDestroy((hipEvent_t)s.done);
        if (s.h_in) (void)hipHostFree(s.h_in);
        if (s.h_out) (void)hipHostFree(s.h_out);
        if (s.d_in) (void)hipFree(s.d_in);
        if (s.d_out) (void)hipFree(s.d_out);
    }
}

Error BatchEncoder::init() {
    fec_ctx* ctx = nullptr;
    Error e = engine_->ctx(&ctx);
    if (!e.ok()) return e;
    const size_t in_bytes = maxBlocks_ * (size_t)k_ * kSlotMax;
    const size_t out_bytes = maxBlocks_ * (size_t)m_ * kSlotMax;
    for (Set& s : sets_) {
        hipError_t h;
        if ((h = hipHostMalloc(&s.h_in, in_bytes, hipHostMallocDefault)) != hipSuccess) return hip_error(h, "hipHostMalloc");
        if ((h = hipHostMalloc(&s.h_out, out_bytes, hipHostMallocDefault)) != hipSuccess) return hip_error(h, "hipHostMalloc");
        if ((h = hipMalloc(&s.d_in, in_bytes)) != hipSuccess) return hip_error(h, "hipMalloc");
        if ((h = hipMalloc(&s.d_out, out_bytes)) != hipSuccess) return hip_error(h, "hipMalloc");
        hipEvent_t ev;
        if ((h = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_error(h, "hipEventCreate");
        s.done = ev;
    }
    ready_ = true;
    return Error::nil();
}

Error BatchEncoder::Submit(Block& b, RepairQueue* q) {
    if (!q) return Error::text("nil repair queue");
    // Validate first (the reference's errors take precedence over any device work), staging
    // into a host scratch slot until the pinned sets exist.
    const size_t want = round16(kRepairPayloadMetadataLen + (size_t)std::max(0, b.biggestSourceSymbolLenSoFar));
    if (!ready_) {
        std::vector<uint8_t> scratch((size_t)std::max(k_, 1) * kSlotMax);
        size_t L = 0;
        int count = 0;
        Error e = rs_ ? rs_->stageRepairInput(b, scratch.data(), kSlotMax, &L)
                      : xor_->stageRepairInput(b, scratch.data(), kSlotMax, &L, &count);
        if (!e.ok()) return e;
        if (xor_ && count != k_) return Error::text("block does not match the encoder's source symbol count");
    }
    Set* s = nullptr;
    Error e = slotFor(want, &s);
    if (!e.ok()) return e;
    uint8_t* dst = s->h_in + s->blocks.size() * (size_t)k_ * s->slot;
    size_t L = 0;
    int count = 0;
    e = rs_ ? rs_->stageRepairInput(b, dst, s->slot, &L) : xor_->stageRepairInput(b, dst, s->slot, &L, &count);
    if (!e.ok()) return e;
    if (xor_ && count != k_) return Error::text("block does not match the encoder's source symbol count");
    s->blocks.push_back(Pending{q, q ? q->token() : nullptr, b.id, L});
    s->maxLen = std::max(s->maxLen, L);
    return Error::nil();
}

// The staging set to write the next block into, with slot >= want (flushes when needed).
// Only device failures fail here: queue backpressure leaves frames in the backlog.
Error BatchEncoder::slotFor(size_t want, Set** out) {
    if (!ready_) {
        Error e = init();
        if (!e.ok()) return e;
    }
    Set* s = &sets_[cur_];
    if (s->inFlight) {
        Error e = retire(*s);
        if (!e.ok()) return e;
    }
    if (!s->blocks.empty() && (s->blocks.size() >= maxBlocks_ || std::max<size_t>(want, 16) > s->slot)) {
        Error e = flushImpl(nullptr);
        if (!e.ok()) return e;
        s = &sets_[cur_];
    }
    if (s->blocks.empty()) s->slot = std::min(kSlotMax, std::max<size_t>(want, 16));
    *out = s;
    return Error::nil();
}

Error BatchEncoder::SubmitPayloads(BlockID id, const uint8_t* const* payloads, const size_t* lens, int count,
                                   RepairQueue* q) {
    if (count < 0 || (count && (!payloads || !lens))) return Error::text("invalid payload list");
    // repairSymbols' checks for a block holding exactly these payloads: complete (reed_solomon.go:27,
    // xor.go:15) -> (XOR: one repair symbol) -> size (reed_solomon.go:31, xor.go:23)
    if (count != k_) return errIncomplete();
    size_t biggest = 0;
    for (int i = 0; i < count; ++i) biggest = std::max(biggest, lens[i]);
    if (biggest > kMaxFECPacketBufferSize) return errTooBig((int)biggest);
    const size_t L = biggest + kRepairPayloadMetadataLen;
    Set* s = nullptr;
    Error e = slotFor(round16(L), &s);
    if (!e.ok()) return e;
    uint8_t* dst = s->h_in + s->blocks.size() * (size_t)k_ * s->slot;
    for (int i = 0; i < count; ++i) {
        uint8_t* slot = dst + (size_t)i * s->slot;
        if (lens[i]) memcpy(slot, payloads[i], lens[i]);
        memset(slot + lens[i], 0, round16(L) - lens[i]);
        // RS: big-endian length trailer at [biggest] (reed_solomon.go:77-87); XOR: the same
        // BE16 XORed in (xor.go:49-53), which for one framed payload is the same bytes
        slot[biggest] = (uint8_t)(lens[i] >> 8);
        slot[biggest + 1] = (uint8_t)(lens[i] & 0xFF);
    }
    s->blocks.push_back(Pending{q, q ? q->token() : nullptr, id, L});
    s->maxLen = std::max(s->maxLen, L);
    return Error::nil();
}

Error BatchEncoder::Flush() { return flushImpl(nullptr); }

bool BatchEncoder::PopRaw(RawBlock* out) {
    if (raw_.empty()) return false;
    *out = std::move(raw_.front());
    raw_.pop_front();
    return true;
}

Error BatchEncoder::flushImpl(size_t* delivered) {
    Set& s = sets_[cur_];
    if (s.inFlight) {
        Error e = retire(s);
        if (!e.ok()) return e;
    }
    if (s.blocks.empty()) return Error::nil();
    fec_ctx* ctx = nullptr;
    Error e = engine_->ctx(&ctx);
    if (!e.ok()) return e;
    hipStream_t st = (hipStream_t)fec_ctx_stream(ctx);
    const size_t B = s.blocks.size();
    hipError_t h = hipMemcpyAsync(s.d_in, s.h_in, B * (size_t)k_ * s.slot, hipMemcpyHostToDevice, st);
    if (h != hipSuccess) return hip_error(h, "hipMemcpyAsync H2D");
    int rc;
    if (rs_)
        rc = fec_rs_encode_batch(ctx, k_, m_, s.maxLen, B, s.d_in, (size_t)k_ * s.slot, s.d_out, (size_t)m_ * s.slot,
                                 s.slot, FEC_DEVICE);
    else
        rc = fec_xor_encode_batch(ctx, k_, s.maxLen, B, s.d_in, (size_t)k_ * s.slot, s.d_out, s.slot, s.slot,
                                  FEC_DEVICE);
    if (rc) return codec_rc(rc);
    if ((h = hipMemcpyAsync(s.h_out, s.d_out, B * (size_t)m_ * s.slot, hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_error(h, "hipMemcpyAsync D2H");
    if ((h = hipEventRecord((hipEvent_t)s.done, st)) != hipSuccess) return hip_error(h, "hipEventRecord");
    s.inFlight = true;
    cur_ ^= 1;
    // the other set becomes the staging set: retire it if its batch is still out
    Set& next = sets_[cur_];
    if (next.inFlight) {
        if (!(e = retire(next)).ok()) return e;
    }
    pump(delivered);   // a full queue is not a failure of this flush
    return Error::nil();
}

Error BatchEncoder::waitSet(Set& s) {
    const hipError_t h = hipEventSynchronize((hipEvent_t)s.done);
    return h == hipSuccess ? Error::nil() : hip_error(h, "hipEventSynchronize");
}

Error BatchEncoder::retire(Set& s) {
    Error e = waitSet(s);
    if (!e.ok()) return e;
    for (size_t i = 0; i < s.blocks.size(); ++i) {
        const Pending& p = s.blocks[i];
        if (!p.q) {   // no queue: keep the payloads, back to back, for PopRaw
            RawBlock rb;
            rb.id = p.id;
            rb.len = p.len;
            rb.bytes.resize((size_t)m_ * p.len);
            for (int j = 0; j < m_; ++j)
                memcpy(rb.bytes.data() + (size_t)j * p.len, s.h_out + (i * (size_t)m_ + j) * s.slot, p.len);
            raw_.push_back(std::move(rb));
            continue;
        }
        Ready r{p.q, p.tok, p.id, {}};
        r.payloads.reserve((size_t)m_);
        for (int j = 0; j < m_; ++j) {
            // repairSymbols makes RS payloads as make([]byte, 0, MaxPacketBufferSize)[:L']
            // (reed_solomon.go:44-49) and the XOR payload as make([]byte, L) (xor.go:28-33)
            Slice pl = rs_ ? Slice::make(0, kMaxPacketBufferSize).reslice(0, p.len) : Slice::make(p.len, p.len);
            memcpy(pl.data(), s.h_out + (i * (size_t)m_ + j) * s.slot, p.len);
            r.payloads.push_back(pl);
        }
        backlog_.push_back(std::move(r));
    }
    s.blocks.clear();
    s.maxLen = 0;
    s.inFlight = false;
    return Error::nil();
}

bool BatchEncoder::pump(size_t* blocks) {
    std::vector<RepairQueue*> held;   // queues whose next block did not fit: keep their order
    for (auto it = backlog_.begin(); it != backlog_.end();) {
        if (std::find(held.begin(), held.end(), it->q) != held.end()) {
            ++it;
            continue;
        }
        std::lock_guard<std::mutex> lk(it->tok->mu);   // the queue cannot be freed meanwhile
        // a freed or closed queue drops its frames, as the reference's closed connection would
        if (it->tok->alive && !it->q->Closed()) {
            if (it->q->Len() + it->payloads.size() > it->q->MaxLen()) {
                held.push_back(it->q);
                ++it;
                continue;
            }
            for (size_t j = 0; j < it->payloads.size(); ++j)
                (void)it->q->Add(RepairFrame{it->id, (ParityID)j, it->payloads[j]});
            if (blocks) ++*blocks;
        }
        it = backlog_.erase(it);
    }
    return backlog_.empty();
}

Error BatchEncoder::Poll(size_t* blocks) {
    if (blocks) *blocks = 0;
    // the older batch is the one not being staged
    for (int i = 1; i >= 0; --i) {
        Set& s = sets_[cur_ ^ i];
        if (!s.inFlight) continue;
        const hipError_t h = hipEventQuery((hipEvent_t)s.done);
        if (h == hipErrorNotReady) break;   // later batches complete later (one stream)
        if (h != hipSuccess) return hip_error(h, "hipEventQuery");
        Error e = retire(s);
        if (!e.ok()) return e;
    }
    return pump(blocks) ? Error::nil() : Error::text("repair queue full");
}

Error BatchEncoder::Drain(size_t* blocks) {
    if (blocks) *blocks = 0;
    size_t n = 0;
    Error e = flushImpl(&n);
    if (!e.ok()) return e;
    for (int i = 1; i >= 0; --i) {
        Set& s = sets_[cur_ ^ i];
        if (!s.inFlight) continue;
        if (!(e = retire(s)).ok()) return e;
    }
    const bool empty = pump(&n);
    if (blocks) *blocks = n;
    return empty ? Error::nil() : Error::text("repair queue full");
}

size_t BatchEncoder::Staged() const { return sets_[cur_].blocks.size(); }

size_t BatchEncoder::InFlight() const {
    const Set& o = sets_[cur_ ^ 1];
    return o.inFlight ? o.blocks.size() : 0;
}

size_t BatchEncoder::Backlog() const { return backlog_.size(); }

}  // namespace fec

namespace fec {

// ------------------------------------------------------------------ RecoveredQueue

void RecoveredQueue::Push(Item it) {
    std::lock_guard<std::mutex> lk(mu_);
    q_.push_back(std::move(it));
}

bool RecoveredQueue::Pop(Item* out) {
    std::lock_guard<std::mutex> lk(mu_);
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    return true;
}

size_t RecoveredQueue::Len() {
    std::lock_guard<std::mutex> lk(mu_);
    return q_.size();
}

// ------------------------------------------------------------------ BatchDecoder

Error BatchDecoder::New(DecoderFECScheme scheme, int k, int m, size_t maxBlocks, std::shared_ptr<Engine> engine,
                        std::unique_ptr<BatchDecoder>* out) {
    out->reset();
    if (maxBlocks == 0) return Error::text("batch must hold at least one block");
    std::unique_ptr<BatchDecoder> d(new BatchDecoder(scheme, k, m, maxBlocks, std::move(engine)));
    if (scheme == ReedSolomonFECScheme) {
        Error err = ReedSolomonScheme::New(k, m, d->engine_, &d->rs_);
        if (!err.ok()) return err;
        if (k + m > FEC_MAX_DECODE_SHARDS) return codec_rc(FEC_ERR_MAX_SHARD_NUM);
    } else if (scheme == XORFECScheme) {
        if (m != 1) return Error::text("xor only supports 1 repair symbol");
        if (k < 1 || k > 255) return Error::text("invalid number of source symbols");
        d->xor_.reset(new XorScheme(d->engine_));
    } else {
        return Error::text("no FEC scheme");
    }
    *out = std::move(d);
    return Error::nil();
}

BatchDecoder::~BatchDecoder() {
    for (Set& s : sets_) {
        if (s.inFlight && s.done) (void)hipEventSynchronize((hipEvent_t)s.done);
        if (s.done) (void)hipEventDestroy((hipEvent_t)s.done);
        for (void* p : {(void*)s.h_in, (void*)s.h_out, (void*)s.h_masks, (void*)s.h_status})
            if (p) (void)hipHostFree(p);
        for (void* p : {(void*)s.d_in, (void*)s.d_out, (void*)s.d_masks, (void*)s.d_status})
            if (p) (void)hipFree(p);
    }
}

Error BatchDecoder::init() {
    fec_ctx* ctx = nullptr;
    Error e = engine_->ctx(&ctx);
    if (!e.ok()) return e;
    const size_t n = (size_t)k_ + m_;
    const size_t in_bytes = maxBlocks_ * n * kDecSlotMax, out_bytes = maxBlocks_ * (size_t)m_ * kDecSlotMax;
    for (Set& s : sets_) {
        hipError_t h;
        if ((h = hipHostMalloc(&s.h_in, in_bytes, hipHostMallocDefault)) != hipSuccess ||
            (h = hipHostMalloc(&s.h_out, out_bytes, hipHostMallocDefault)) != hipSuccess ||
            (h = hipHostMalloc(&s.h_masks, maxBlocks_ * 4, hipHostMallocDefault)) != hipSuccess ||
            (h = hipHostMalloc(&s.h_status, maxBlocks_ * 4, hipHostMallocDefault)) != hipSuccess ||
            (h = hipMalloc(&s.d_in, in_bytes)) != hipSuccess || (h = hipMalloc(&s.d_out, out_bytes)) != hipSuccess ||
            (h = hipMalloc(&s.d_masks, maxBlocks_ * 4)) != hipSuccess ||
            (h = hipMalloc(&s.d_status, maxBlocks_ * 4)) != hipSuccess)
            return hip_error(h, "staging allocation");
        hipEvent_t ev;
        if ((h = hipEventCreateWithFlags(&ev, hipEventDisableTiming)) != hipSuccess) return hip_error(h, "hipEventCreate");
        s.done = ev;
    }
    ready_ = true;
    return Error::nil();
}

Error BatchDecoder::stage(Block& b, uint8_t* dst, size_t slot, Pending* p, bool* nothing) {
    *nothing = false;
    p->id = b.id;
    p->meta = Block{};
    p->meta.id = b.id;
    p->meta.totNumSourceSymbols = b.totNumSourceSymbols;
    p->meta.totNumRepairSymbols = b.totNumRepairSymbols;
    p->meta.smallestSSID = b.smallestSSID;
    p->meta.largestSSID = b.largestSSID;
    p->meta.biggestSourceSymbolLenSoFar = b.biggestSourceSymbolLenSoFar;
    if (rs_) {
        Error e = rs_->stageRecoverInput(b, dst, slot, &p->plan);
        if (!e.ok()) return e;
        *nothing = p->plan.nothing;
        return Error::nil();
    }
    int count = 0;
    Error e = xor_->stageRecoverInput(b, dst, slot, (size_t)k_, nothing, &count);
    if (!e.ok()) return e;
    p->plan = ReedSolomonScheme::RecoverPlan{};
    p->plan.len = slot;
    return Error::nil();
}

template <class StageFn>
Error BatchDecoder::submitWith(size_t want, RecoveredQueue* q, bool* staged, StageFn&& stage_fn) {
    if (staged) *staged = false;
    if (!q) return Error::text("nil recovered queue");
    want = std::min(kDecSlotMax, std::max<size_t>(16, round16(want)));
    const size_t n = (size_t)k_ + m_;
    bool nothing = false;
    Pending p;
    if (!ready_) {   // validate before any device work
        std::vector<uint8_t> scratch(n * kDecSlotMax);
        Error e = stage_fn(scratch.data(), kDecSlotMax, &p, &nothing);
        if (!e.ok() || nothing) return e;
        if (!(e = init()).ok()) return e;
    }
    Set* s = &sets_[cur_];
    if (s->inFlight) {
        Error e = waitSet(*s);
        if (e.ok()) e = deliver(*s, nullptr);
        if (!e.ok()) return e;
    }
    if (!s->blocks.empty() && (s->blocks.size() >= maxBlocks_ || want > s->slot)) {
        Error e = flushImpl(nullptr);
        if (!e.ok()) return e;
        s = &sets_[cur_];
    }
    if (s->blocks.empty()) s->slot = want;
    const size_t idx = s->blocks.size();
    Error e = stage_fn(s->h_in + idx * n * s->slot, s->slot, &p, &nothing);
    if (!e.ok() || nothing) return e;
    s->h_masks[idx] = p.plan.mask;
    s->maxLen = std::max(s->maxLen, rs_ ? p.plan.len : s->slot);
    s->outSlots = std::max(s->outSlots, rs_ ? p.plan.missing.size() : (size_t)1);
    p.q = q;
    p.tok = q->token();
    s->blocks.push_back(std::move(p));
    if (staged) *staged = true;
    return Error::nil();
}

Error BatchDecoder::Submit(Block& b, RecoveredQueue* q, bool* staged) {
    size_t want = kRepairPayloadMetadataLen + (size_t)std::max(0, b.biggestSourceSymbolLenSoFar);
    for (auto& kv : b.pidToRepairPayload) want = std::max(want, kv.second.len);
    return submitWith(want, q, staged, [&](uint8_t* dst, size_t slot, Pending* p, bool* nothing) {
        return stage(b, dst, slot, p, nothing);
    });
}

Error BatchDecoder::SubmitPayloads(BlockID id, SourceSymbolID smallest, SourceSymbolID largest, int biggest,
                                   const uint8_t* const* src, const size_t* slen, const uint8_t* const* rep,
                                   const size_t* rlen, RecoveredQueue* q, bool* staged) {
    if (staged) *staged = false;
    if (!src || !slen || !rep || !rlen) return Error::text("invalid payload list");
    size_t want = kRepairPayloadMetadataLen + (size_t)std::max(0, biggest);
    for (int p = 0; p < m_; ++p)
        if (rep[p]) want = std::max(want, rlen[p]);
    return submitWith(want, q, staged, [&](uint8_t* dst, size_t slot, Pending* p, bool* nothing) {
        *nothing = false;
        p->id = id;
        p->meta = Block{};
        p->meta.id = id;
        p->meta.totNumSourceSymbols = k_;
        p->meta.totNumRepairSymbols = m_;
        p->meta.smallestSSID = smallest;
        p->meta.largestSSID = largest;
        p->meta.biggestSourceSymbolLenSoFar = biggest;
        if (rs_) {
            Error e = rs_->stageRecoverPayloads(biggest, src, slen, rep, rlen, dst, slot, &p->plan);
            if (e.ok()) *nothing = p->plan.nothing;
            return e;
        }
        int count = 0;
        Error e = xor_->stageRecoverPayloads(k_, m_, biggest, src, slen, rep, rlen, dst, slot, (size_t)k_, nothing,
                                             &count);
        p->plan = ReedSolomonScheme::RecoverPlan{};
        p->plan.len = slot;
        return e;
    });
}

Error BatchDecoder::Flush() { return flushImpl(nullptr); }

Error BatchDecoder::flushImpl(size_t* delivered) {
    Set& s = sets_[cur_];
    if (s.inFlight) {
        Error e = waitSet(s);
        if (e.ok()) e = deliver(s, delivered);
        if (!e.ok()) return e;
    }
    if (s.blocks.empty()) return Error::nil();
    fec_ctx* ctx = nullptr;
    Error e = engine_->ctx(&ctx);
    if (!e.ok()) return e;
    hipStream_t st = (hipStream_t)fec_ctx_stream(ctx);
    const size_t B = s.blocks.size(), n = (size_t)k_ + m_, S = s.slot;
    const size_t nin = rs_ ? n : (size_t)k_;   // XOR stages its k inputs only
    hipError_t h = hipMemcpyAsync(s.d_in, s.h_in, B * n * S, hipMemcpyHostToDevice, st);
    if (h != hipSuccess) return hip_error(h, "hipMemcpyAsync H2D");
    int rc;
    if (rs_) {
        if ((h = hipMemcpyAsync(s.d_masks, s.h_masks, B * 4, hipMemcpyHostToDevice, st)) != hipSuccess)
            return hip_error(h, "hipMemcpyAsync H2D");
        rc = fec_rs_recover_batch(ctx, k_, m_, s.maxLen, B, s.d_in, n * S, s.d_in + (size_t)k_ * S, n * S, S,
                                  s.d_masks, s.d_out, s.outSlots * S, (int)s.outSlots, s.d_status, FEC_DEVICE);
    } else {
        rc = fec_xor_encode_batch(ctx, (int)nin, s.maxLen, B, s.d_in, n * S, s.d_out, S, S, FEC_DEVICE);
    }
    if (rc) return codec_rc(rc);
    if ((h = hipMemcpyAsync(s.h_out, s.d_out, B * s.outSlots * S, hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_error(h, "hipMemcpyAsync D2H");
    if (rs_ && (h = hipMemcpyAsync(s.h_status, s.d_status, B * 4, hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_error(h, "hipMemcpyAsync D2H");
    if ((h = hipEventRecord((hipEvent_t)s.done, st)) != hipSuccess) return hip_error(h, "hipEventRecord");
    s.inFlight = true;
    s.delivered = 0;
    cur_ ^= 1;
    Set& next = sets_[cur_];
    if (next.inFlight) {
        if ((e = waitSet(next)).ok()) e = deliver(next, delivered);
        if (!e.ok()) return e;
    }
    return Error::nil();
}

Error BatchDecoder::waitSet(Set& s) {
    const hipError_t h = hipEventSynchronize((hipEvent_t)s.done);
    return h == hipSuccess ? Error::nil() : hip_error(h, "hipEventSynchronize");
}

Error BatchDecoder::deliver(Set& s, size_t* blocks) {
    const size_t B = s.blocks.size(), S = s.slot;
    for (; s.delivered < B; ++s.delivered) {
        Pending& p = s.blocks[s.delivered];
        Slice out;
        Error e;
        if (rs_) {
            if (s.h_status[s.delivered] != (int32_t)p.plan.missing.size())
                return codec_rc(s.h_status[s.delivered] < 0 ? s.h_status[s.delivered] : FEC_ERR_HIP);
            std::vector<const uint8_t*> rebuilt;
            for (size_t r = 0; r < p.plan.missing.size(); ++r)
                rebuilt.push_back(s.h_out + (s.delivered * s.outSlots + r) * S);
            e = rs_->finishRecover(p.meta, p.plan, rebuilt.data(), &out);
        } else {
            e = xor_->finishRecover(p.meta, s.h_out + s.delivered * S, S, &out);
        }
        if (!e.ok()) return e;
        std::lock_guard<std::mutex> lk(p.tok->mu);
        if (p.tok->alive) {   // a freed queue (its connection closed) drops the block
            p.q->Push(RecoveredQueue::Item{p.id, out});
            if (blocks) ++*blocks;
        }
    }
    s.blocks.clear();
    s.maxLen = s.outSlots = s.delivered = 0;
    s.inFlight = false;
    return Error::nil();
}

Error BatchDecoder::Poll(size_t* blocks) {
    if (blocks) *blocks = 0;
    for (int i = 1; i >= 0; --i) {
        Set& s = sets_[cur_ ^ i];
        if (!s.inFlight) continue;
        const hipError_t h = hipEventQuery((hipEvent_t)s.done);
        if (h == hipErrorNotReady) break;
        if (h != hipSuccess) return hip_error(h, "hipEventQuery");
        Error e = deliver(s, blocks);
        if (!e.ok()) return e;
    }
    return Error::nil();
}

Error BatchDecoder::Drain(size_t* blocks) {
    size_t before = 0;
    Error e = flushImpl(&before);
    if (blocks) *blocks = 0;
    if (!e.ok()) return e;
    for (int i = 1; i >= 0; --i) {
        Set& s = sets_[cur_ ^ i];
        if (!s.inFlight) continue;
        if (!(e = waitSet(s)).ok()) return e;
        size_t n = 0;
        if (!(e = deliver(s, &n)).ok()) return e;
        before += n;
    }
    if (blocks) *blocks = before;
    return Error::nil();
}

size_t BatchDecoder::Staged() const { return sets_[cur_].blocks.size(); }

size_t BatchDecoder::InFlight() const {
    const Set& o = sets_[cur_ ^ 1];
    return o.inFlight ? o.blocks.size() - o.delivered : 0;
}

}  // namespace fec
