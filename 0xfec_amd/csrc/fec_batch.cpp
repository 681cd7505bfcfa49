// fec_batch.cpp — RepairQueue (repair_queue.go restated) and BatchEncoder (deferred, batched
// repair-symbol generation on the GPU). Design and contracts: include/fec_batch.hpp.
#include "../../include/fec_batch.hpp"

#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/fec_hip.h"
#include "fec_kernels.hpp"

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

// ------------------------------------------------------------------ PacketPool

namespace {
struct PoolEntry {
    uintptr_t lo, hi;
    uint64_t dev;
    std::weak_ptr<PacketPool> pool;
};
std::mutex g_pool_mu;
std::vector<PoolEntry> g_pools;
}  // namespace

Error PacketPool::New(size_t nbuf, std::shared_ptr<PacketPool>* out) {
    out->reset();
    if (nbuf == 0 || nbuf > (size_t(1) << 26)) return Error::text("packet pool size out of range");
    std::shared_ptr<PacketPool> p(new PacketPool());
    p->bytes_ = nbuf * kSlot;
    void* base = nullptr;
    hipError_t h = hipHostMalloc(&base, p->bytes_, hipHostMallocMapped | hipHostMallocPortable);
    if (h != hipSuccess) return hip_error(h, "hipHostMalloc");
    p->base_ = static_cast<uint8_t*>(base);
    memset(p->base_, 0, p->bytes_);
    void* dev = nullptr;
    if ((h = hipHostGetDevicePointer(&dev, base, 0)) != hipSuccess) return hip_error(h, "hipHostGetDevicePointer");
    p->dev_ = (uint64_t)(uintptr_t)dev;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pools.push_back(PoolEntry{(uintptr_t)p->base_, (uintptr_t)p->base_ + p->bytes_, p->dev_, p});
    }
    *out = std::move(p);
    return Error::nil();
}

PacketPool::~PacketPool() {
    Unregister();
    if (base_) (void)hipHostFree(base_);
}

void PacketPool::Unregister() {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto it = g_pools.begin(); it != g_pools.end(); ++it)
        if (it->lo == (uintptr_t)base_) {
            g_pools.erase(it);
            break;
        }
}

uint64_t PacketPool::Lookup(const uint8_t* p, size_t len, std::shared_ptr<PacketPool>* pool) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (const PoolEntry& e : g_pools)
        if (a >= e.lo && a <= e.hi && len <= e.hi - a) {   // the same test as DevAddr
            std::shared_ptr<PacketPool> sp = e.pool.lock();
            if (!sp) return 0;
            *pool = std::move(sp);
            return e.dev + (a - e.lo);
        }
    return 0;
}

// ------------------------------------------------------------------ BatchEncoder

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
        if (s.h_desc) (void)hipHostFree(s.h_desc);
        if (s.d_desc) (void)hipFree(s.d_desc);
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
        const size_t desc_bytes = maxBlocks_ * (size_t)k_ * sizeof(fk::GatherDesc);
        if ((h = hipHostMalloc(&s.h_desc, desc_bytes, hipHostMallocDefault)) != hipSuccess)
            return hip_error(h, "hipHostMalloc");
        if ((h = hipMalloc(&s.d_desc, desc_bytes)) != hipSuccess) return hip_error(h, "hipMalloc");
        void *in_dev = nullptr, *out_dev = nullptr, *desc_dev = nullptr;
        if ((h = hipHostGetDevicePointer(&in_dev, s.h_in, 0)) != hipSuccess ||
            (h = hipHostGetDevicePointer(&out_dev, s.h_out, 0)) != hipSuccess ||
            (h = hipHostGetDevicePointer(&desc_dev, s.h_desc, 0)) != hipSuccess)
            return hip_error(h, "hipHostGetDevicePointer");
        s.in_dev = (uint64_t)(uintptr_t)in_dev;
        s.out_dev = static_cast<uint8_t*>(out_dev);
        s.desc_dev = desc_dev;
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
    // the framed shards as gather descriptors too, in case a referenced block joins this batch
    fk::GatherDesc* desc = static_cast<fk::GatherDesc*>(s->h_desc) + s->blocks.size() * (size_t)k_;
    for (int i = 0; i < k_; ++i)
        desc[i] = fk::GatherDesc{s->in_dev + (uint64_t)(dst - s->h_in) + (uint64_t)i * s->slot, (uint32_t)L, fk::kNoFrame};
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
    if (holding_ == cur_) spill(*s);
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
    Set* s = nullptr;
    Error e = slotFor(round16(biggest + kRepairPayloadMetadataLen), &s);
    if (!e.ok()) return e;
    return stageBlock(s, id, payloads, lens, biggest, false, q);
}

Error BatchEncoder::SubmitRefs(BlockID id, const uint8_t* const* payloads, const size_t* lens, int count,
                               RepairQueue* q) {
    if (count < 0 || (count && (!payloads || !lens))) return Error::text("invalid payload list");
    if (count != k_) return errIncomplete();   // the same checks, in the same order, as SubmitPayloads
    size_t biggest = 0;
    for (int i = 0; i < count; ++i) biggest = std::max(biggest, lens[i]);
    if (biggest > kMaxFECPacketBufferSize) return errTooBig((int)biggest);
    Set* s = nullptr;
    Error e = slotFor(round16(biggest + kRepairPayloadMetadataLen), &s);
    if (!e.ok()) return e;
    return stageBlock(s, id, payloads, lens, biggest, true, q);
}

// One validated block into set s: each payload either framed into its pinned slot here, or (refs,
// and it lies in a registered pool) left where it is, to be gathered and framed by the device.
// Every shard gets a gather descriptor, so a batch is gathered as a whole once any shard needs it.
Error BatchEncoder::stageBlock(Set* s, BlockID id, const uint8_t* const* payloads, const size_t* lens, size_t biggest,
                               bool refs, RepairQueue* q) {
    const size_t L = biggest + kRepairPayloadMetadataLen;
    uint8_t* dst = s->h_in + s->blocks.size() * (size_t)k_ * s->slot;
    fk::GatherDesc* desc = static_cast<fk::GatherDesc*>(s->h_desc) + s->blocks.size() * (size_t)k_;
    for (int i = 0; i < k_; ++i) {
        if (refs && lens[i]) {
            // the pools this batch already holds first (no lock, no reference count traffic: the
            // senders of many connections share one pool), the registry only on a miss
            uint64_t dev = 0;
            for (const auto& pool : s->pools)
                if ((dev = pool->DevAddr(payloads[i], lens[i]))) break;
            if (!dev) {
                std::shared_ptr<PacketPool> pool;
                if ((dev = PacketPool::Lookup(payloads[i], lens[i], &pool))) s->pools.push_back(std::move(pool));
            }
            if (dev) {
                desc[i] = fk::GatherDesc{dev, (uint32_t)lens[i], (uint32_t)biggest};
                s->gather = true;
                continue;
            }
        }
        uint8_t* slot = dst + (size_t)i * s->slot;
        if (lens[i]) memcpy(slot, payloads[i], lens[i]);
        memset(slot + lens[i], 0, round16(L) - lens[i]);
        // RS: big-endian length trailer at [biggest] (reed_solomon.go:77-87); XOR: the same
        // BE16 XORed in (xor.go:49-53), which for one framed payload is the same bytes
        slot[biggest] = (uint8_t)(lens[i] >> 8);
        slot[biggest + 1] = (uint8_t)(lens[i] & 0xFF);
        desc[i] = fk::GatherDesc{s->in_dev + (uint64_t)(slot - s->h_in), (uint32_t)L, fk::kNoFrame};
    }
    s->blocks.push_back(Pending{q, q ? q->token() : nullptr, id, L});
    s->maxLen = std::max(s->maxLen, L);
    return Error::nil();
}

Error BatchEncoder::Flush() { return flushImpl(nullptr); }

bool BatchEncoder::PeekRaw(RawView* out) {
    if (!raw_.empty()) {
        const RawBlock& r = raw_.front();
        *out = RawView{r.id, r.len, r.bytes.data(), r.len};
        return true;
    }
    if (holding_ < 0) return false;
    const Set& s = sets_[holding_];
    const Pending& p = s.blocks[s.rawNext];
    *out = RawView{p.id, p.len, s.h_out + s.rawNext * (size_t)m_ * s.slot, s.slot};
    return true;
}

void BatchEncoder::PopRaw() {
    if (!raw_.empty()) {
        raw_.pop_front();
        return;
    }
    if (holding_ < 0) return;
    Set& s = sets_[holding_];
    if (++s.rawNext < s.blocks.size()) return;
    s.blocks.clear();
    s.maxLen = 0;
    s.rawNext = 0;
    holding_ = -1;
}

size_t BatchEncoder::RawLen() const {
    return raw_.size() + (holding_ >= 0 ? sets_[holding_].blocks.size() - sets_[holding_].rawNext : 0);
}

void BatchEncoder::spill(Set& s) {
    for (size_t i = s.rawNext; i < s.blocks.size(); ++i) {
        const Pending& p = s.blocks[i];
        RawBlock rb;
        rb.id = p.id;
        rb.len = p.len;
        rb.bytes.resize((size_t)m_ * p.len);
        for (int j = 0; j < m_; ++j)
            memcpy(rb.bytes.data() + (size_t)j * p.len, s.h_out + (i * (size_t)m_ + j) * s.slot, p.len);
        raw_.push_back(std::move(rb));
    }
    s.blocks.clear();
    s.maxLen = 0;
    s.rawNext = 0;
    holding_ = -1;
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
    hipError_t h;
    // a small set is coded straight from and into its pinned buffers: one launch (two when
    // gathered) and an event instead of a copy up, the launch, a copy down (knob bat_zc, as the
    // decoder's sets)
    const bool zc = B * (size_t)k_ * s.slot <= (size_t)std::max(0, (int)fk::g_tune.bat_zc);
    uint8_t* in = zc ? reinterpret_cast<uint8_t*>((uintptr_t)s.in_dev) : s.d_in;
    uint8_t* out = zc ? s.out_dev : s.d_out;
    if (s.gather) {   // referenced payloads: the device pulls every shard of the batch itself
        const void* desc = s.desc_dev;
        if (!zc) {
            if ((h = hipMemcpyAsync(s.d_desc, s.h_desc, B * (size_t)k_ * sizeof(fk::GatherDesc), hipMemcpyHostToDevice,
                                    st)) != hipSuccess)
                return hip_error(h, "hipMemcpyAsync H2D");
            desc = s.d_desc;
        }
        if ((h = hipSetDevice(engine_->device())) != hipSuccess) return hip_error(h, "hipSetDevice");
        if ((h = fk::launch_gather_desc(static_cast<const fk::GatherDesc*>(desc), (uint32_t)(B * (size_t)k_), s.d_in,
                                        s.slot, st)) != hipSuccess)
            return hip_error(h, "gather launch");
        in = s.d_in;
    } else if (!zc &&
               (h = hipMemcpyAsync(s.d_in, s.h_in, B * (size_t)k_ * s.slot, hipMemcpyHostToDevice, st)) != hipSuccess) {
        return hip_error(h, "hipMemcpyAsync H2D");
    }
    int rc;
    if (rs_)
        rc = fec_rs_encode_batch(ctx, k_, m_, s.maxLen, B, in, (size_t)k_ * s.slot, out, (size_t)m_ * s.slot, s.slot,
                                 FEC_DEVICE);
    else
        rc = fec_xor_encode_batch(ctx, k_, s.maxLen, B, in, (size_t)k_ * s.slot, out, s.slot, s.slot, FEC_DEVICE);
    if (rc) return codec_rc(rc);
    if (!zc && (h = hipMemcpyAsync(s.h_out, s.d_out, B * (size_t)m_ * s.slot, hipMemcpyDeviceToHost, st)) != hipSuccess)
        return hip_error(h, "hipMemcpyAsync D2H");
    if ((h = hipEventRecord((hipEvent_t)s.done, st)) != hipSuccess) return hip_error(h, "hipEventRecord");
    s.inFlight = true;
    cur_ ^= 1;
    // the other set becomes the staging set: retire it if its batch is still out
    Set& next = sets_[cur_];
    if (next.inFlight) {
        if (!(e = retire(next)).ok()) return e;
    }
    if (holding_ == cur_) spill(next);
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
    s.pools.clear();   // the device has read every referenced payload
    s.gather = false;
    s.inFlight = false;
    bool raw_only = !s.blocks.empty();
    for (const Pending& p : s.blocks) raw_only = raw_only && !p.q;
    const int idx = (int)(&s - sets_);
    // an older holding set's blocks go out before any of this set's: raw_ only ever holds blocks
    // older than a holding set's (PeekRaw serves raw_ first)
    if (holding_ >= 0 && holding_ != idx) spill(sets_[holding_]);
    if (raw_only) {   // hand the blocks out of h_out in place (PeekRaw)
        holding_ = idx;
        s.rawNext = 0;
        return Error::nil();
    }
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
        // Our own reference to the token: when the queue is gone, the backlog entry may hold the
        // last one, and erasing the entry must not free the mutex this scope still holds.
        const std::shared_ptr<QueueToken> tok = it->tok;
        {
            std::lock_guard<std::mutex> lk(tok->mu);   // the queue cannot be freed meanwhile
            // a freed or closed queue drops its frames, as the reference's closed connection would
            if (tok->alive && !it->q->Closed()) {
                if (it->q->Len() + it->payloads.size() > it->q->MaxLen()) {
                    held.push_back(it->q);
                    ++it;
                    continue;
                }
                for (size_t j = 0; j < it->payloads.size(); ++j)
                    (void)it->q->Add(RepairFrame{it->id, (ParityID)j, it->payloads[j]});
                if (blocks) ++*blocks;
            }
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
        for (void* p : {(void*)s.h_in, (void*)s.h_out, (void*)s.h_masks, (void*)s.h_status, s.h_desc})
            if (p) (void)hipHostFree(p);
        for (void* p : {(void*)s.d_in, (void*)s.d_out, (void*)s.d_masks, (void*)s.d_status, s.d_desc})
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
            (h = hipMalloc(&s.d_status, maxBlocks_ * 4)) != hipSuccess ||
            (h = hipHostMalloc(&s.h_desc, maxBlocks_ * n * sizeof(fk::GatherDesc), hipHostMallocDefault)) != hipSuccess ||
            (h = hipMalloc(&s.d_desc, maxBlocks_ * n * sizeof(fk::GatherDesc))) != hipSuccess)
            return hip_error(h, "staging allocation");
        void *in_dev = nullptr, *out_dev = nullptr, *masks_dev = nullptr, *status_dev = nullptr, *desc_dev = nullptr;
        if ((h = hipHostGetDevicePointer(&in_dev, s.h_in, 0)) != hipSuccess ||
            (h = hipHostGetDevicePointer(&out_dev, s.h_out, 0)) != hipSuccess ||
            (h = hipHostGetDevicePointer(&masks_dev, s.h_masks, 0)) != hipSuccess ||
            (h = hipHostGetDevicePointer(&status_dev, s.h_status, 0)) != hipSuccess ||
            (h = hipHostGetDevicePointer(&desc_dev, s.h_desc, 0)) != hipSuccess)
            return hip_error(h, "hipHostGetDevicePointer");
        s.in_dev = (uint64_t)(uintptr_t)in_dev;
        s.out_dev = static_cast<uint8_t*>(out_dev);
        s.masks_dev = static_cast<uint32_t*>(masks_dev);
        s.status_dev = static_cast<int32_t*>(status_dev);
        s.desc_dev = desc_dev;
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
Error BatchDecoder::submitWith(size_t want, RecoveredQueue* q, bool* staged, StageFn&& stage_fn,
                               const ShardRef* refs, std::vector<std::shared_ptr<PacketPool>>* pools) {
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
    // every shard of the block gets a gather descriptor (its staged slot unless referenced), so a
    // set is gathered as a whole once any block of it holds a reference
    fk::GatherDesc* desc = static_cast<fk::GatherDesc*>(s->h_desc) + idx * n;
    for (size_t i = 0; i < n; ++i) {
        if (refs && refs[i].dev) {
            desc[i] = fk::GatherDesc{refs[i].dev, refs[i].len, refs[i].frame};
            s->gather = true;
        } else {
            desc[i] = fk::GatherDesc{s->in_dev + (uint64_t)((idx * n + i) * s->slot), (uint32_t)s->slot, fk::kNoFrame};
        }
    }
    if (pools)
        for (auto& pl : *pools)
            if (std::find(s->pools.begin(), s->pools.end(), pl) == s->pools.end()) s->pools.push_back(pl);
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

Error BatchDecoder::SubmitPayloadRefs(BlockID id, SourceSymbolID smallest, SourceSymbolID largest, int biggest,
                                      const uint8_t* const* src, const size_t* slen, const uint8_t* const* rep,
                                      const size_t* rlen, RecoveredQueue* q, bool* staged) {
    if (!rs_ || !src || !slen || !rep || !rlen || biggest < 0)
        return SubmitPayloads(id, smallest, largest, biggest, src, slen, rep, rlen, q, staged);
    if (staged) *staged = false;
    // the shards the device can gather: a source within `biggest` (a longer one is cut at biggest
    // + 2 on the host, addLengthToSourceSymbolPayload's reslice) or a repair, in a registered pool
    const size_t n = (size_t)k_ + m_;
    std::vector<ShardRef> refs(n, ShardRef{0, 0, 0});
    std::vector<uint8_t> skip(n, 0);
    std::vector<std::shared_ptr<PacketPool>> pools;
    for (size_t i = 0; i < n; ++i) {
        const bool isSrc = i < (size_t)k_;
        const uint8_t* ptr = isSrc ? src[i] : rep[i - k_];
        const size_t len = isSrc ? slen[i] : rlen[i - k_];
        if (!ptr || len == 0 || (isSrc && len > (size_t)biggest)) continue;
        uint64_t dev = 0;
        for (const auto& pl : pools)
            if ((dev = pl->DevAddr(ptr, len))) break;
        if (!dev) {
            std::shared_ptr<PacketPool> pl;
            if ((dev = PacketPool::Lookup(ptr, len, &pl))) pools.push_back(std::move(pl));
        }
        if (!dev) continue;
        refs[i] = ShardRef{dev, (uint32_t)len, isSrc ? (uint32_t)biggest : fk::kNoFrame};
        skip[i] = 1;
    }
    size_t want = kRepairPayloadMetadataLen + (size_t)biggest;
    for (int p = 0; p < m_; ++p)
        if (rep[p]) want = std::max(want, rlen[p]);
    return submitWith(
        want, q, staged,
        [&](uint8_t* dst, size_t slot, Pending* p, bool* nothing) {
            *nothing = false;
            p->id = id;
            p->meta = Block{};
            p->meta.id = id;
            p->meta.totNumSourceSymbols = k_;
            p->meta.totNumRepairSymbols = m_;
            p->meta.smallestSSID = smallest;
            p->meta.largestSSID = largest;
            p->meta.biggestSourceSymbolLenSoFar = biggest;
            Error e = rs_->stageRecoverPayloads(biggest, src, slen, rep, rlen, dst, slot, &p->plan,
                                                reinterpret_cast<const bool*>(skip.data()));
            if (e.ok()) *nothing = p->plan.nothing;
            return e;
        },
        refs.data(), &pools);
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
    hipError_t h;
    // a small set (a receive burst of a few blocks) is coded straight from and into its pinned
    // buffers: one launch (two when gathered) and an event, where the copy form makes four copies
    // around the kernels, each a call of its own and a copy-engine round trip (knob bat_zc: input
    // bytes up to which; go_batch_bench burst)
    const bool zc = B * n * S <= (size_t)std::max(0, (int)fk::g_tune.bat_zc);
    uint8_t* in = zc ? reinterpret_cast<uint8_t*>((uintptr_t)s.in_dev) : s.d_in;
    uint8_t* out = zc ? s.out_dev : s.d_out;
    uint32_t* masks = zc ? s.masks_dev : s.d_masks;
    int32_t* status = zc ? s.status_dev : s.d_status;
    if (s.gather) {   // referenced payloads: the device pulls every shard of the set itself
        const void* desc = s.desc_dev;
        if (!zc) {
            if ((h = hipMemcpyAsync(s.d_desc, s.h_desc, B * n * sizeof(fk::GatherDesc), hipMemcpyHostToDevice, st)) !=
                hipSuccess)
                return hip_error(h, "hipMemcpyAsync H2D");
            desc = s.d_desc;
        }
        if ((h = hipSetDevice(engine_->device())) != hipSuccess) return hip_error(h, "hipSetDevice");
        if ((h = fk::launch_gather_desc(static_cast<const fk::GatherDesc*>(desc), (uint32_t)(B * n), s.d_in, S, st)) !=
            hipSuccess)
            return hip_error(h, "gather launch");
        in = s.d_in;
    } else if (!zc && (h = hipMemcpyAsync(s.d_in, s.h_in, B * n * S, hipMemcpyHostToDevice, st)) != hipSuccess) {
        return hip_error(h, "hipMemcpyAsync H2D");
    }
    int rc;
    if (rs_) {
        if (!zc && (h = hipMemcpyAsync(s.d_masks, s.h_masks, B * 4, hipMemcpyHostToDevice, st)) != hipSuccess)
            return hip_error(h, "hipMemcpyAsync H2D");
        rc = fec_rs_recover_batch(ctx, k_, m_, s.maxLen, B, in, n * S, in + (size_t)k_ * S, n * S, S, masks, out,
                                  s.outSlots * S, (int)s.outSlots, status, FEC_DEVICE);
    } else {
        rc = fec_xor_encode_batch(ctx, (int)nin, s.maxLen, B, in, n * S, out, S, S, FEC_DEVICE);
    }
    if (rc) return codec_rc(rc);
    if (!zc) {
        if ((h = hipMemcpyAsync(s.h_out, s.d_out, B * s.outSlots * S, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_error(h, "hipMemcpyAsync D2H");
        if (rs_ && (h = hipMemcpyAsync(s.h_status, s.d_status, B * 4, hipMemcpyDeviceToHost, st)) != hipSuccess)
            return hip_error(h, "hipMemcpyAsync D2H");
    }
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
    s.gather = false;
    s.pools.clear();
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
