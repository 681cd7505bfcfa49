// fec_batch.hpp — the sender-side batching layer the GPU needs.
//
// In the reference, repair symbols are generated synchronously, one block at a time, inside
// the packet packer (packet_packer.go:1001-1011 -> manager.go:145 -> reed_solomon.go:51), and
// queued per connection in a 32-frame ring (repair_queue.go:17-99). A GPU launch per block
// costs more than the reference's whole per-block encode, so here the encode is deferred:
//
//   RepairQueue   repair_queue.go restated (Add / Peek / Pop / CloseWithError, hasData
//                 callback, the 32-frame limit). The reference panics when full; the mirror
//                 returns the error "repair queue full" instead. The limit is a constructor
//                 argument because a batch delivers many blocks' frames at once.
//   BatchEncoder  collects complete blocks from any number of connections (each with its own
//                 RepairQueue) into pinned staging, [block][k][S] with S = the batch's 16-byte
//                 slot; Flush() issues one H2D copy, one encode launch and one D2H copy on the
//                 encoder's stream and returns; Poll() hands the repair frames of completed
//                 batches to their queues in submission order. Two staging sets: a batch
//                 stages while the previous one is in flight.
//
// Frames are bit-identical to the per-block path: a block's repair payload is the first
// L = biggest + 2 bytes of its parity shards, and zero padding of the other blocks of the
// batch (shard_len = the batch's largest L) does not change those bytes (the code is
// byte-wise). Payloads are made as repairSymbols makes them (make(0, 1452)[:L] for RS,
// make(L, L) for XOR).
#pragma once

#include <stdint.h>

#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <vector>

#include "fec_scheme.hpp"

namespace fec {

// Liveness of a queue that a batch coder holds by pointer until a batch completes: a queue
// freed in the meantime (its connection closed) is marked dead under `mu`, and the coder drops
// that queue's blocks instead of touching the freed object.
struct QueueToken {
    std::mutex mu;
    bool alive = true;
};
inline void kill_token(const std::shared_ptr<QueueToken>& t) {
    std::lock_guard<std::mutex> lk(t->mu);
    t->alive = false;
}

// repair_queue.go:17-99
class RepairQueue {
public:
    static constexpr size_t kMaxRepairSendQueueLen = 32;   // repair_queue.go:14

    explicit RepairQueue(std::function<void()> hasData = nullptr, size_t maxLen = kMaxRepairSendQueueLen)
        : hasData_(std::move(hasData)), maxLen_(maxLen) {}
    ~RepairQueue() { kill_token(token_); }
    RepairQueue(const RepairQueue&) = delete;
    RepairQueue& operator=(const RepairQueue&) = delete;
    const std::shared_ptr<QueueToken>& token() const { return token_; }
    bool Closed();
    // Add queues a new REPAIR frame for sending (repair_queue.go:40-69).
    Error Add(RepairFrame f);
    // Peek gets the next REPAIR frame for sending; nullptr when empty (repair_queue.go:73-80).
    // The pointer stays valid until the next Pop.
    const RepairFrame* Peek();
    // Pop removes the frame Peek returned (repair_queue.go:82-90).
    void Pop();
    // CloseWithError (repair_queue.go:92-95): later Adds return the error.
    void CloseWithError(Error e);
    size_t Len();
    size_t MaxLen() const { return maxLen_; }

private:
    std::mutex mu_;
    std::deque<RepairFrame> q_;
    std::function<void()> hasData_;
    size_t maxLen_;
    bool closed_ = false;
    Error closeErr_;
    std::shared_ptr<QueueToken> token_ = std::make_shared<QueueToken>();
};

// A slab of packet buffers in pinned, device-mapped host memory (the Go ABI's opt-in registered
// pool, include/fec_go.h fec_go_pool_new; the reference allocates each source-symbol payload as
// make([]byte, 0, MaxPacketBufferSize), packet_packer.go:984). A payload built in one of these
// buffers can be handed to BatchEncoder::SubmitRefs by address: the device reads it over PCIe
// when the batch is coded (fec_pack.hip gather_desc_kernel), with no host copy. A pool stays
// alive while any staged batch references it, whatever its owner does meanwhile.
class PacketPool {
public:
    static constexpr size_t kSlot = 1456;   // protocol.MaxPacketBufferSize rounded up to 16 bytes
    static Error New(size_t nbuf, std::shared_ptr<PacketPool>* out);
    ~PacketPool();
    PacketPool(const PacketPool&) = delete;
    PacketPool& operator=(const PacketPool&) = delete;
    uint8_t* base() const { return base_; }
    size_t bytes() const { return bytes_; }
    // Registered pools hold [p, p + len): its device address and the pool, else 0 / null (under
    // the registry's lock: the batch coder asks only for the first payload of each pool per batch).
    static uint64_t Lookup(const uint8_t* p, size_t len, std::shared_ptr<PacketPool>* pool);
    // This pool's device address of [p, p + len), or 0 when the range is not inside it.
    uint64_t DevAddr(const uint8_t* p, size_t len) const {
        const uintptr_t a = (uintptr_t)p, lo = (uintptr_t)base_;
        return (a >= lo && a - lo <= bytes_ && len <= bytes_ - (a - lo)) ? dev_ + (a - lo) : 0;
    }
    // Stop handing this pool out to lookups (the owner is done with it); the memory goes when the
    // last batch referencing it retires.
    void Unregister();

private:
    PacketPool() = default;
    uint8_t* base_ = nullptr;
    uint64_t dev_ = 0;
    size_t bytes_ = 0;
};

class BatchEncoder {
public:
    // scheme: ReedSolomonFECScheme (k, m) or XORFECScheme (k, 1). maxBlocks: blocks per batch.
    static Error New(DecoderFECScheme scheme, int k, int m, size_t maxBlocks, std::shared_ptr<Engine> engine,
                     std::unique_ptr<BatchEncoder>* out);
    ~BatchEncoder();

    // Validate (exactly as repairSymbols: same errors, same order) and stage a complete block;
    // its frames go to q when its batch completes. A full batch, or a block whose shards do not
    // fit the batch's slot, flushes first.
    Error Submit(Block& b, RepairQueue* q);
    // Zero-copy form for integrations that keep their own block bookkeeping (SURVEY.md §8f row
    // 4): the k source payloads of block `id`, in SSID order, framed straight from the caller's
    // packet buffers into pinned staging (one copy; nothing retained after the call, so cgo
    // may pass Go slices). Same checks and errors as repairSymbols for a block holding exactly
    // these payloads.
    // q == nullptr: the block's payloads are kept for PopRaw instead of going to a queue.
    Error SubmitPayloads(BlockID id, const uint8_t* const* payloads, const size_t* lens, int count, RepairQueue* q);
    // By-reference form: a payload lying in a registered PacketPool is not copied, only its
    // address is recorded, and the device gathers and frames it when the batch is coded; the
    // caller keeps it unchanged until the block comes back (PeekRaw / its queue). Any other
    // payload is copied now, as SubmitPayloads. Same checks and errors.
    Error SubmitRefs(BlockID id, const uint8_t* const* payloads, const size_t* lens, int count, RepairQueue* q);
    // Encoded blocks submitted without a queue (the Go ABI, include/fec_go.h, whose caller keeps
    // its own queue), in submission order: repair payload i of the block is len bytes at
    // base + i * stride. The view points into the completed batch's pinned output (no copy) and
    // stays valid until PopRaw or any other call on the encoder.
    struct RawView {
        BlockID id = 0;
        size_t len = 0;
        const uint8_t* base = nullptr;
        size_t stride = 0;
    };
    bool PeekRaw(RawView* out);
    void PopRaw();
    size_t RawLen() const;
    // Start encoding the staged blocks (asynchronous). No-op when nothing is staged.
    Error Flush();
    // Deliver the frames of every completed batch (non-blocking); *blocks = blocks delivered.
    // Frames that do not fit their queue stay in the encoder's backlog (per queue in order)
    // and go out on a later Poll / Drain; the call then returns "repair queue full" (the
    // blocks it did deliver are counted in *blocks all the same). The backlog holds at most
    // the blocks submitted and not yet delivered: it grows only while a queue stays full, and
    // a queue that is closed or freed has its blocks dropped at the next Poll / Drain.
    // Backpressure never fails Submit: a staging set whose frames cannot be delivered yet
    // moves them to the backlog and is reused.
    Error Poll(size_t* blocks = nullptr);
    // Flush, wait for every batch and deliver (backlog as Poll).
    Error Drain(size_t* blocks = nullptr);
    size_t Staged() const;     // blocks staged, not yet flushed
    size_t InFlight() const;   // blocks flushed, not yet encoded and collected
    size_t Backlog() const;    // blocks encoded whose frames wait for room in their queue
    int k() const { return k_; }
    int m() const { return m_; }
    DecoderFECScheme scheme() const { return scheme_; }

private:
    struct Pending {
        RepairQueue* q;
        std::shared_ptr<QueueToken> tok;   // q's liveness (null without a queue)
        BlockID id;
        size_t len;
    };
    struct Set {
        uint8_t* h_in = nullptr;    // pinned [maxBlocks][k][kSlotMax]
        uint8_t* h_out = nullptr;   // pinned [maxBlocks][m][kSlotMax]
        uint8_t* d_in = nullptr;
        uint8_t* d_out = nullptr;
        void* h_desc = nullptr;     // pinned [maxBlocks][k] gather descriptors (fk::GatherDesc)
        void* d_desc = nullptr;
        uint64_t in_dev = 0;        // device address of h_in (pinned, mapped)
        uint8_t* out_dev = nullptr; // h_out and h_desc as the device sees them (small sets are coded
        const void* desc_dev = nullptr;   // straight from and into pinned memory, knob bat_zc)
        void* done = nullptr;       // hipEvent_t
        std::vector<Pending> blocks;
        std::vector<std::shared_ptr<PacketPool>> pools;   // pools the batch's references point into
        size_t slot = 0;            // S of this batch (16-byte multiple)
        size_t maxLen = 0;          // largest L of this batch
        bool gather = false;        // some payload is referenced: the device gathers the batch
        bool inFlight = false;
        size_t rawNext = 0;         // holding (completed, raw blocks kept in h_out): next to hand out
    };
    struct RawBlock {               // a raw block copied out of a set that had to be reused
        BlockID id = 0;
        size_t len = 0;
        std::vector<uint8_t> bytes;
    };
    std::deque<RawBlock> raw_;      // older than any holding set's blocks
    int holding_ = -1;              // the set whose completed raw blocks are handed out in place
    // Copy a holding set's blocks not yet handed out to raw_ and free the set for staging.
    void spill(Set& s);
    Error stageBlock(Set* s, BlockID id, const uint8_t* const* payloads, const size_t* lens, size_t biggest, bool refs,
                     RepairQueue* q);
    struct Ready {                  // an encoded block whose frames wait for queue room
        RepairQueue* q;
        std::shared_ptr<QueueToken> tok;
        BlockID id;
        std::vector<Slice> payloads;   // m repair payloads, ParityID = index
    };
    BatchEncoder(DecoderFECScheme scheme, int k, int m, size_t maxBlocks, std::shared_ptr<Engine> e)
        : scheme_(scheme), k_(k), m_(m), maxBlocks_(maxBlocks), engine_(std::move(e)) {}
    Error init();
    Error flushImpl(size_t* delivered);
    Error waitSet(Set& s);
    // Wait for a flushed set, move its blocks' payloads to the backlog and free the set.
    Error retire(Set& s);
    // Hand backlog frames to their queues in order; a queue that is full holds back its later
    // blocks. *blocks += blocks delivered. True when the backlog is empty afterwards.
    bool pump(size_t* blocks);
    Error slotFor(size_t want, Set** out);

    DecoderFECScheme scheme_;
    int k_, m_;
    size_t maxBlocks_;
    std::shared_ptr<Engine> engine_;
    std::unique_ptr<ReedSolomonScheme> rs_;
    std::unique_ptr<XorScheme> xor_;
    Set sets_[2];
    int cur_ = 0;   // the set being staged
    bool ready_ = false;
    std::deque<Ready> backlog_;
};

// Receive side: recovered payloads of one connection, in the order their
// blocks became recoverable. HandleRepairFrame returns the payload directly in the reference
// (manager.go:160-198, connection.go:1342); batched, it arrives here when the batch completes.
class RecoveredQueue {
public:
    struct Item {
        BlockID block_id;
        Slice payload;   // recoverSymbolPayloads' result (the concatenation, or XOR's payload)
    };
    RecoveredQueue() = default;
    ~RecoveredQueue() { kill_token(token_); }
    RecoveredQueue(const RecoveredQueue&) = delete;
    RecoveredQueue& operator=(const RecoveredQueue&) = delete;
    void Push(Item it);
    bool Pop(Item* out);   // false when empty
    size_t Len();
    const std::shared_ptr<QueueToken>& token() const { return token_; }

private:
    std::mutex mu_;
    std::deque<Item> q_;
    std::shared_ptr<QueueToken> token_ = std::make_shared<QueueToken>();
};

// Deferred, batched recoverSymbolPayloads: recoverable blocks of any number of connections are
// staged into pinned memory ([block][n][S], present shards + present masks), decoded with one
// H2D copy, one fec_rs_recover_batch (or XOR) launch and one D2H copy per batch, and their
// payloads handed to each block's RecoveredQueue in submission order. Two staging sets.
class BatchDecoder {
public:
    static Error New(DecoderFECScheme scheme, int k, int m, size_t maxBlocks, std::shared_ptr<Engine> engine,
                     std::unique_ptr<BatchDecoder>* out);
    ~BatchDecoder();
    // Validate (exactly as recoverSymbolPayloads: same errors, same order) and stage a
    // recoverable block. A block that is already complete is the reference's nil, nil: nothing
    // is staged or delivered (*staged = false).
    Error Submit(Block& b, RecoveredQueue* q, bool* staged = nullptr);
    // Zero-copy form for integrations that keep their own block bookkeeping (the Go binding,
    // include/fec_go.h): the block's SSID range, biggest and payload pointers (src: k entries,
    // SSID smallest + i; rep: m entries, ParityID p; nullptr = absent), validated and framed
    // straight into pinned staging with the same checks, errors and order as Submit. Nothing is
    // retained after the call.
    Error SubmitPayloads(BlockID id, SourceSymbolID smallest, SourceSymbolID largest, int biggest,
                         const uint8_t* const* src, const size_t* slen, const uint8_t* const* rep, const size_t* rlen,
                         RecoveredQueue* q, bool* staged = nullptr);
    // By-reference form (RS): a present payload lying in a registered PacketPool is validated but
    // not copied; the device gathers it (sources framed with their BE16 length trailer at
    // `biggest`, repairs verbatim) when the batch is coded. Others are staged as by
    // SubmitPayloads; XOR decoders stage everything. The pool buffers must stay unchanged until
    // the block comes back from Poll / Drain.
    Error SubmitPayloadRefs(BlockID id, SourceSymbolID smallest, SourceSymbolID largest, int biggest,
                            const uint8_t* const* src, const size_t* slen, const uint8_t* const* rep,
                            const size_t* rlen, RecoveredQueue* q, bool* staged = nullptr);
    Error Flush();
    Error Poll(size_t* blocks = nullptr);
    Error Drain(size_t* blocks = nullptr);
    size_t Staged() const;
    size_t InFlight() const;
    DecoderFECScheme scheme() const { return scheme_; }

private:
    struct Pending {
        RecoveredQueue* q;
        std::shared_ptr<QueueToken> tok;   // q's liveness
        BlockID id;
        Block meta;                // id, biggest, SSID range (payload maps not kept)
        ReedSolomonScheme::RecoverPlan plan;   // RS: mask, length, missing indices
    };
    struct Set {
        uint8_t* h_in = nullptr;    // pinned [maxBlocks][n][kDecSlotMax]
        uint8_t* h_out = nullptr;   // pinned [maxBlocks][m][kDecSlotMax]
        uint32_t* h_masks = nullptr;
        int32_t* h_status = nullptr;
        uint8_t* d_in = nullptr;
        uint8_t* d_out = nullptr;
        uint32_t* d_masks = nullptr;
        int32_t* d_status = nullptr;
        void* done = nullptr;
        std::vector<Pending> blocks;
        size_t slot = 0, maxLen = 0, outSlots = 0, delivered = 0;
        bool inFlight = false;
        void* h_desc = nullptr;     // pinned [maxBlocks][n] gather descriptors (fk::GatherDesc)
        void* d_desc = nullptr;
        uint64_t in_dev = 0;        // h_in as the device sees it
        // the other pinned buffers as the device sees them (small sets are coded straight from and
        // into pinned memory: no copy engine round trips, fewer calls per flush)
        uint8_t* out_dev = nullptr;
        uint32_t* masks_dev = nullptr;
        int32_t* status_dev = nullptr;
        const void* desc_dev = nullptr;
        bool gather = false;        // a block of the set is referenced: the device gathers the set
        std::vector<std::shared_ptr<PacketPool>> pools;   // pools the set's references point into
    };
    BatchDecoder(DecoderFECScheme scheme, int k, int m, size_t maxBlocks, std::shared_ptr<Engine> e)
        : scheme_(scheme), k_(k), m_(m), maxBlocks_(maxBlocks), engine_(std::move(e)) {}
    Error init();
    Error stage(Block& b, uint8_t* dst, size_t slot, Pending* p, bool* nothing);
    // Submit's body: `stage_fn(dst, slot, &pending, &nothing)` validates and stages one block;
    // refs (nullable, n entries): shards left where they are (dev != 0) for the device to gather
    struct ShardRef {
        uint64_t dev;              // device-visible address, 0: the shard is staged
        uint32_t len, frame;       // bytes, BE16 trailer position (or fk::kNoFrame)
    };
    template <class StageFn>
    Error submitWith(size_t want, RecoveredQueue* q, bool* staged, StageFn&& stage_fn,
                     const ShardRef* refs = nullptr, std::vector<std::shared_ptr<PacketPool>>* pools = nullptr);
    Error flushImpl(size_t* delivered);
    Error waitSet(Set& s);
    Error deliver(Set& s, size_t* blocks);

    DecoderFECScheme scheme_;
    int k_, m_;
    size_t maxBlocks_;
    std::shared_ptr<Engine> engine_;
    std::unique_ptr<ReedSolomonScheme> rs_;
    std::unique_ptr<XorScheme> xor_;
    Set sets_[2];
    int cur_ = 0;
    bool ready_ = false;
};

}  // namespace fec
