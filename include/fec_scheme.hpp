// fec_scheme.hpp — C++ mirror of the reference's internal/fec scheme and manager layer.
//
// ddritzenhoff/0xFEC keeps its block bookkeeping in Go (internal/fec/block.go,
// manager.go) and its arithmetic in klauspost/reedsolomon + Go byte loops
// (reed_solomon.go, xor.go). The Go toolchain is absent from this build image, so the
// layer above the C ABI is restated here in C++ with the same names, argument meaning,
// error texts and error ordering; the arithmetic goes through lib0xfec_hip.so
// (include/fec_hip.h) on the GPU. A Go integration keeps its own Go code and binds only
// fec_hip.h; this mirror is what the parity tests drive.
//
// Go slices are modelled by Slice (shared backing array, len, cap) because the reference
// relies on slice aliasing: addLengthToSourceSymbolPayload writes the length trailer into
// the payload's spare capacity (reed_solomon.go:70-89) and xorScheme.recoverSymbolPayloads
// stores the recovered slice into the block map (xor.go:91-96).
#pragma once

#include <stdint.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

struct fec_ctx;

namespace fec {

// internal/protocol/protocol.go:111,136-140
constexpr size_t kMaxPacketBufferSize = 1452;
constexpr size_t kMaxFECHeaderOverhead = 18;
constexpr size_t kMaxFECPacketBufferSize = kMaxPacketBufferSize - kMaxFECHeaderOverhead;   // 1434
constexpr size_t kRepairPayloadMetadataLen = 2;

// internal/protocol/fec.go:8-27
using SourceSymbolID = uint64_t;
using BlockID = uint64_t;
using ParityID = uint64_t;
enum DecoderFECScheme : uint8_t { FECDisabled = 0, XORFECScheme = 1, ReedSolomonFECScheme = 2 };

// A Go []byte: a window [off, off+len) of a shared backing array with capacity cap.
struct Slice {
    std::shared_ptr<std::vector<uint8_t>> buf;
    size_t off = 0, len = 0, cap = 0;

    static Slice make(size_t len, size_t cap);                    // make([]byte, len, cap), zeroed
    static Slice from(const uint8_t* p, size_t len, size_t cap);  // copy of p, spare capacity zeroed
    bool nil() const { return !buf; }
    uint8_t* data() { return buf ? buf->data() + off : nullptr; }
    const uint8_t* data() const { return buf ? buf->data() + off : nullptr; }
    Slice reslice(size_t lo, size_t hi) const;                    // s[lo:hi], hi <= cap
    std::vector<uint8_t> bytes() const { return std::vector<uint8_t>(data(), data() + len); }
};

// A Go error: ok() when nil.
struct Error {
    std::string msg;
    int code = 0;   // 0: scheme/bookkeeping error (msg); < 0: fec_hip.h codec code
    bool ok() const { return msg.empty() && code == 0; }
    static Error nil() { return Error{}; }
    static Error text(std::string m) { return Error{std::move(m), 0}; }
};

// internal/wire/fec_repair_frame.go:11-14, fec_source_symbol_frame.go:11-17
struct RepairFrame {
    BlockID block_id = 0;
    ParityID parity_id = 0;
    Slice payload;
};

struct SourceSymbolFrame {
    SourceSymbolID ssid = 0;
    Slice payload;
};

// internal/fec/block.go:23-95
struct Block {
    BlockID id = 0;
    std::map<SourceSymbolID, Slice> ssidToSourcePayload;
    std::map<ParityID, Slice> pidToRepairPayload;
    SourceSymbolID smallestSSID = 0, largestSSID = 0;
    int totNumSourceSymbols = 0;
    int totNumRepairSymbols = 0;
    int biggestSourceSymbolLenSoFar = 0;

    static Block New(BlockID id, int totNumSourceSymbols, int totNumRepairSymbols);   // newBlock
    Error addSourceSymbol(const SourceSymbolFrame& f);
    Error addRepairSymbol(const RepairFrame& f);
    bool isRecoverable() const;
    bool isComplete() const;
};

// The reference's error values shared with the batching layer (reed_solomon.go:28,32).
Error errIncomplete();
Error errTooBig(int biggest);

// internal/fec/scheme.go:5-10
class BlockFECScheme {
public:
    virtual ~BlockFECScheme() = default;
    virtual Error repairSymbols(Block& b, std::vector<RepairFrame>* out) = 0;
    // *out stays nil (Slice::nil()) when the reference returns nil, nil.
    virtual Error recoverSymbolPayloads(Block& b, Slice* out) = 0;
};

// Device binding shared by the schemes of one process thread: one fec_ctx per device,
// created on first compute (a scheme can be built and validated without a GPU).
class Engine {
public:
    explicit Engine(int device) : device_(device) {}
    ~Engine();
    Error ctx(fec_ctx** out);
    int device() const { return device_; }

private:
    int device_;
    fec_ctx* ctx_ = nullptr;
};

// internal/fec/reed_solomon.go:11-136 (klauspost Encode/ReconstructData -> HIP kernels)
class ReedSolomonScheme : public BlockFECScheme {
public:
    // NewReedSolomonScheme (reed_solomon.go:15-23); klauspost New validation.
    static Error New(int numTotSourceSymbols, int numTotRepairSymbols, std::shared_ptr<Engine> engine,
                     std::unique_ptr<ReedSolomonScheme>* out);
    Error repairSymbols(Block& b, std::vector<RepairFrame>* out) override;
    Error recoverSymbolPayloads(Block& b, Slice* out) override;
    int dataShards() const { return k_; }
    int parityShards() const { return m_; }
    // repairSymbols up to the enc.Encode call (same checks, same errors, same order): writes the
    // block's k framed shards to dst + i*stride (zero pad to the 16-byte boundary) and their
    // length L. The batch encoder (fec_batch.hpp) stages blocks with it.
    Error stageRepairInput(Block& b, uint8_t* dst, size_t stride, size_t* shard_len);
    // recoverSymbolPayloads up to the enc.ReconstructData call (same checks, same order): the
    // present shards into dst + i*stride (n slots), the present mask, shard length and missing
    // data indices; plan->nothing when the block is already complete (nil result).
    struct RecoverPlan {
        bool nothing = false;
        size_t len = 0;
        uint32_t mask = 0;
        std::vector<int> missing;   // ascending missing data shard indices
    };
    Error stageRecoverInput(Block& b, uint8_t* dst, size_t stride, RecoverPlan* plan);
    // The same for a block given as its payloads (fec_go_decoder_submit: no Block built):
    // src[i] = the payload of SSID smallestSSID + i or nullptr, read with the capacity of a
    // packet buffer (kMaxPacketBufferSize); rep[p] = the payload of ParityID p or nullptr.
    // skip (nullable, k + m entries): shard i is validated and counted but not written (the
    // caller has the device gather it, BatchDecoder::SubmitPayloadRefs).
    Error stageRecoverPayloads(int biggest, const uint8_t* const* src, const size_t* slen, const uint8_t* const* rep,
                               const size_t* rlen, uint8_t* dst, size_t stride, RecoverPlan* plan,
                               const bool* skip = nullptr);
    // The rest of recoverSymbolPayloads: rebuilt[r] = the rebuilt shard of plan.missing[r].
    Error finishRecover(const Block& b, const RecoverPlan& plan, const uint8_t* const* rebuilt, Slice* out);

private:
    ReedSolomonScheme(int k, int m, std::shared_ptr<Engine> e) : k_(k), m_(m), engine_(std::move(e)) {}
    Error addLengthToSourceSymbolPayload(Block& b, SourceSymbolID ssid, Slice* out);
    int k_, m_;
    std::shared_ptr<Engine> engine_;
};

// internal/fec/xor.go:10-104 (byte loops -> HIP XOR kernel)
class XorScheme : public BlockFECScheme {
public:
    explicit XorScheme(std::shared_ptr<Engine> engine) : engine_(std::move(engine)) {}
    Error repairSymbols(Block& b, std::vector<RepairFrame>* out) override;
    Error recoverSymbolPayloads(Block& b, Slice* out) override;
    // repairSymbols up to the XOR reduction: the sources framed (payload, BE16 length XORed at
    // [biggest]) into dst + i*stride, their count and length L.
    Error stageRepairInput(Block& b, uint8_t* dst, size_t stride, size_t* shard_len, int* count);
    // recoverSymbolPayloads up to the XOR loop (same checks): repairs and framed sources into
    // `slots` slots of `stride` bytes (unused slots zeroed); *nothing when already complete.
    Error stageRecoverInput(Block& b, uint8_t* dst, size_t stride, size_t slots, bool* nothing, int* count);
    // The same for a block given as its k source / m repair payload pointers (nullptr absent).
    Error stageRecoverPayloads(int k, int m, int biggest, const uint8_t* const* src, const size_t* slen,
                               const uint8_t* const* rep, const size_t* rlen, uint8_t* dst, size_t stride,
                               size_t slots, bool* nothing, int* count);
    // The rest of recoverSymbolPayloads from the XOR of the inputs (len bytes of it).
    Error finishRecover(Block& b, const uint8_t* rec, size_t len, Slice* out);

private:
    std::shared_ptr<Engine> engine_;
};

// internal/fec/manager.go:13-227
class Manager {
public:
    static Error New(std::unique_ptr<BlockFECScheme> scheme, int numTotSourceSymbols, int numTotRepairSymbols,
                     std::unique_ptr<Manager>* out);
    SourceSymbolID NextSSID();
    Error AddSourceSymbolFrame(const SourceSymbolFrame& f, std::vector<RepairFrame>* out);
    Error HandleRepairFrame(const RepairFrame& f, Slice* out);
    // manager.go:200-227. `recovered` (optional) receives the payloads recovered because this
    // source made the block recoverable; only with SetRecoverOnSource(true), else it stays nil.
    Error HandleSourceSymbolFrame(const SourceSymbolFrame& f, Slice* out, Slice* recovered = nullptr);
    // Off by default (reference behaviour): recovery fires only on a REPAIR arrival
    // (manager.go:181), so a block whose repairs arrived before its k-th surviving source is
    // never recovered (manager.go:221-226 only checks isComplete). On: a source arrival that
    // makes the block recoverable but not complete recovers it too.
    void SetRecoverOnSource(bool on) { recoverOnSource_ = on; }
    bool RecoverOnSource() const { return recoverOnSource_; }
    BlockID sidToBlockID(SourceSymbolID sid) const;
    size_t trackedBlocks() const { return blockStatuses_.size(); }
    // AddSourceSymbolFrame with the encode deferred to a batch: on the k-th source symbol the
    // block is staged into `enc` (validated exactly as repairSymbols would), dropped and marked
    // processed; its repair frames reach `q` when the batch completes (fec_batch.hpp).
    Error AddSourceSymbolFrameBatched(const SourceSymbolFrame& f, class BatchEncoder* enc, class RepairQueue* q);
    // HandleRepairFrame with the recovery deferred to a batch: when the block becomes
    // recoverable it is staged into `dec`, dropped and marked processed; its recovered payload
    // reaches `q` when the batch completes.
    Error HandleRepairFrameBatched(const RepairFrame& f, class BatchDecoder* dec, class RecoveredQueue* q);
    // HandleSourceSymbolFrame (the payload is returned in *out, as there) with the
    // recover-on-source recovery, when enabled, deferred to `dec` like HandleRepairFrameBatched.
    Error HandleSourceSymbolFrameBatched(const SourceSymbolFrame& f, Slice* out, class BatchDecoder* dec,
                                         class RecoveredQueue* q);
    BlockFECScheme* scheme() { return scheme_.get(); }

private:
    struct BlockStatus {
        std::unique_ptr<Block> block;
        bool isProcessed = false;
    };
    BlockStatus& statusFor(BlockID id);
    std::unique_ptr<BlockFECScheme> scheme_;
    std::mutex nextSIDMutex_;
    SourceSymbolID nextSID_ = 0;
    int numTotSourceSymbols_ = 0;
    int numTotRepairSymbols_ = 0;
    std::map<BlockID, BlockStatus> blockStatuses_;
    bool recoverOnSource_ = false;
};

// manager.go:50-94: XOR -> (2,1), ReedSolomon -> (20,10); FECDisabled -> nil manager, nil error.
Error NewSender(DecoderFECScheme id, std::shared_ptr<Engine> engine, std::unique_ptr<Manager>* out);
Error NewReceiver(DecoderFECScheme id, std::shared_ptr<Engine> engine, std::unique_ptr<Manager>* out);

}  // namespace fec
