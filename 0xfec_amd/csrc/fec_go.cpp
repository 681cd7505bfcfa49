// fec_go.cpp — the batched C ABI for the Go package (include/fec_go.h) over the batching layer
// (fec_batch.hpp): payloads come in one pointer per call and are copied at once, complete and
// recoverable blocks are coded in batches, results go out into caller-owned buffers.
#include "../../include/fec_go.h"

#include <string.h>

#include <limits>
#include <map>
#include <memory>
#include <vector>

#include "../../include/fec_batch.hpp"
#include "../../include/fec_hip.h"

namespace fec {
namespace cabi {
int report(const fec::Error& e);
}  // namespace cabi
}  // namespace fec

using fec::cabi::report;

// Each encoder / decoder owns its Engine (its own fec_ctx: stream, workspace, sticky error).
// The Go side makes one per connection and drives it from that connection's run loop
// (connection.go:525), whose goroutine migrates between OS threads: a ctx shared per OS thread
// (fec_scheme.cpp engine_for) would be driven by two connections at once from two threads.
static std::shared_ptr<fec::Engine> own_engine(int device) { return std::make_shared<fec::Engine>(device); }

struct fec_go_encoder {
    int k = 0, m = 0;
    std::unique_ptr<fec::BatchEncoder> enc;   // blocks go in without a queue (PopRaw)
    struct Building {
        std::vector<std::vector<uint8_t>> payload;
        std::vector<bool> have;
    };
    std::map<uint64_t, Building> building;   // blocks whose payloads are being added
};

struct fec_go_decoder {
    int k = 0, m = 0;
    std::unique_ptr<fec::BatchDecoder> dec;
    fec::RecoveredQueue q;
    std::map<uint64_t, fec::Block> blocks;   // block.go state of blocks not yet committed
};

static fec::DecoderFECScheme scheme_of(int id) {
    return id == FEC_SCHEME_XOR ? fec::XORFECScheme : id == FEC_SCHEME_REED_SOLOMON ? fec::ReedSolomonFECScheme
                                                                                      : fec::FECDisabled;
}

extern "C" {

fec_go_encoder* fec_go_encoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int* err) {
    std::unique_ptr<fec_go_encoder> e(new fec_go_encoder());
    e->k = k;
    e->m = scheme_id == FEC_SCHEME_XOR ? 1 : m;
    const int rc = report(fec::BatchEncoder::New(scheme_of(scheme_id), k, m, max_blocks, own_engine(device), &e->enc));
    if (err) *err = rc;
    return rc ? nullptr : e.release();
}

void fec_go_encoder_free(fec_go_encoder* e) { delete e; }

int fec_go_encoder_add(fec_go_encoder* e, uint64_t block_id, int index, const uint8_t* payload, size_t len) {
    if (!e || index < 0 || index >= e->k || (len && !payload))
        return report(fec::Error::text("source payload index outside the block"));
    if (len > fec::kMaxPacketBufferSize) return report(fec::Error::text("source payload longer than a packet buffer"));
    auto& b = e->building[block_id];
    if (b.payload.empty()) {
        b.payload.resize((size_t)e->k);
        b.have.assign((size_t)e->k, false);
    }
    if (!b.have[(size_t)index]) {   // block.go:63: a duplicate SSID is ignored
        b.payload[(size_t)index].assign(payload, payload + len);
        b.have[(size_t)index] = true;
    }
    return FEC_OK;
}

int fec_go_encoder_commit(fec_go_encoder* e, uint64_t block_id) {
    if (!e) return FEC_ERR_INVALID_ARG;
    auto it = e->building.find(block_id);
    std::vector<const uint8_t*> ptrs;
    std::vector<size_t> lens;
    if (it != e->building.end())
        for (size_t i = 0; i < it->second.payload.size(); ++i)
            if (it->second.have[i]) {
                ptrs.push_back(it->second.payload[i].data());
                lens.push_back(it->second.payload[i].size());
            }
    const int rc = report(e->enc->SubmitPayloads(block_id, ptrs.data(), lens.data(), (int)ptrs.size(), nullptr));
    if (it != e->building.end()) e->building.erase(it);
    return rc;
}

int fec_go_encoder_submit(fec_go_encoder* e, uint64_t block_id, const uint8_t* const* payloads, const size_t* lens,
                          int count) {
    if (!e) return FEC_ERR_INVALID_ARG;
    return report(e->enc->SubmitPayloads(block_id, payloads, lens, count, nullptr));
}

int fec_go_encoder_submit_ref(fec_go_encoder* e, uint64_t block_id, const uint8_t* const* payloads,
                              const size_t* lens, int count) {
    if (!e) return FEC_ERR_INVALID_ARG;
    return report(e->enc->SubmitRefs(block_id, payloads, lens, count, nullptr));
}

struct fec_go_pool {
    std::shared_ptr<fec::PacketPool> p;
};

fec_go_pool* fec_go_pool_new(size_t nbuf, uint8_t** base, int* err) {
    if (base) *base = nullptr;
    std::unique_ptr<fec_go_pool> gp(new fec_go_pool());
    const int rc = report(fec::PacketPool::New(nbuf, &gp->p));
    if (err) *err = rc;
    if (rc) return nullptr;
    if (base) *base = gp->p->base();
    return gp.release();
}

void fec_go_pool_free(fec_go_pool* p) {
    if (!p) return;
    p->p->Unregister();   // no new references; the memory goes with the last batch that reads it
    delete p;
}

int fec_go_encoder_flush(fec_go_encoder* e) { return e ? report(e->enc->Flush()) : FEC_ERR_INVALID_ARG; }

int fec_go_encoder_poll(fec_go_encoder* e, int wait, uint64_t* block_ids, uint32_t* repair_len, uint8_t* repairs,
                        size_t max_blocks, size_t* nblocks) {
    if (nblocks) *nblocks = 0;
    if (!e || (max_blocks && (!block_ids || !repair_len || !repairs))) return FEC_ERR_INVALID_ARG;
    fec::Error err = wait ? e->enc->Drain() : e->enc->Poll();
    // start coding the staged blocks when the device has no batch of this encoder in flight:
    // a block never waits for a full batch, and batches grow while the previous one is out
    if (err.ok() && !wait && e->enc->InFlight() == 0 && e->enc->Staged() > 0) err = e->enc->Flush();
    if (!err.ok()) return report(err);
    size_t d = 0;
    fec::BatchEncoder::RawView rv;
    for (; d < max_blocks && e->enc->PeekRaw(&rv); ++d, e->enc->PopRaw()) {   // one copy, out of pinned memory
        block_ids[d] = rv.id;
        repair_len[d] = (uint32_t)rv.len;
        const size_t c = std::min(rv.len, (size_t)FEC_GO_SLOT);
        for (int i = 0; i < e->m; ++i)
            memcpy(repairs + (d * (size_t)e->m + (size_t)i) * FEC_GO_SLOT, rv.base + (size_t)i * rv.stride, c);
    }
    if (nblocks) *nblocks = d;
    return report(fec::Error::nil());
}

fec_go_decoder* fec_go_decoder_new(int scheme_id, int k, int m, size_t max_blocks, int device, int* err) {
    std::unique_ptr<fec_go_decoder> d(new fec_go_decoder());
    d->k = k;
    d->m = scheme_id == FEC_SCHEME_XOR ? 1 : m;
    const int rc = report(fec::BatchDecoder::New(scheme_of(scheme_id), k, m, max_blocks, own_engine(device), &d->dec));
    if (err) *err = rc;
    return rc ? nullptr : d.release();
}

void fec_go_decoder_free(fec_go_decoder* d) { delete d; }

static fec::Block& block_of(fec_go_decoder* d, uint64_t block_id) {
    auto it = d->blocks.find(block_id);
    if (it == d->blocks.end()) it = d->blocks.emplace(block_id, fec::Block::New(block_id, d->k, d->m)).first;
    return it->second;
}

int fec_go_decoder_add_source(fec_go_decoder* d, uint64_t block_id, uint64_t ssid, const uint8_t* payload,
                              size_t len) {
    if (!d || (len && !payload)) return FEC_ERR_INVALID_ARG;
    if (len > fec::kMaxPacketBufferSize) return report(fec::Error::text("source payload longer than a packet buffer"));
    // the receiver's source payloads sit in packet buffers: cap 1452, zeroed (fec_source_symbol_frame.go:34)
    return report(block_of(d, block_id).addSourceSymbol(
        fec::SourceSymbolFrame{ssid, fec::Slice::from(payload, len, fec::kMaxPacketBufferSize)}));
}

int fec_go_decoder_add_repair(fec_go_decoder* d, uint64_t block_id, uint64_t parity_id, const uint8_t* payload,
                              size_t len) {
    if (!d || (len && !payload)) return FEC_ERR_INVALID_ARG;
    // a repair payload's capacity is its length (fec_repair_frame.go:36)
    return report(block_of(d, block_id).addRepairSymbol(
        fec::RepairFrame{block_id, parity_id, fec::Slice::from(payload, len, len)}));
}

int fec_go_decoder_commit(fec_go_decoder* d, uint64_t block_id, int* staged) {
    if (staged) *staged = 0;
    if (!d) return FEC_ERR_INVALID_ARG;
    auto it = d->blocks.find(block_id);
    if (it == d->blocks.end()) return report(fec::Error::text("unknown block"));
    bool st = false;
    const int rc = report(d->dec->Submit(it->second, &d->q, &st));
    if (staged) *staged = st ? 1 : 0;
    if (rc == FEC_OK) d->blocks.erase(it);
    return rc;
}

int fec_go_decoder_submit(fec_go_decoder* d, uint64_t block_id, uint64_t smallest_ssid, uint64_t largest_ssid,
                          int biggest, const uint8_t* const* sources, const size_t* source_lens,
                          const uint8_t* const* repairs, const size_t* repair_lens, int* staged) {
    if (staged) *staged = 0;
    if (!d || !sources || !source_lens || !repairs || !repair_lens) return FEC_ERR_INVALID_ARG;
    for (int i = 0; i < d->k; ++i)
        if (sources[i] && source_lens[i] > fec::kMaxPacketBufferSize)
            return report(fec::Error::text("source payload longer than a packet buffer"));
    bool st = false;
    const int rc = report(d->dec->SubmitPayloads(block_id, smallest_ssid, largest_ssid, biggest, sources, source_lens,
                                                  repairs, repair_lens, &d->q, &st));
    if (staged) *staged = st ? 1 : 0;
    return rc;
}

int fec_go_decoder_submit_ref(fec_go_decoder* d, uint64_t block_id, uint64_t smallest_ssid, uint64_t largest_ssid,
                              int biggest, const uint8_t* const* sources, const size_t* source_lens,
                              const uint8_t* const* repairs, const size_t* repair_lens, int* staged) {
    if (staged) *staged = 0;
    if (!d || !sources || !source_lens || !repairs || !repair_lens) return FEC_ERR_INVALID_ARG;
    for (int i = 0; i < d->k; ++i)
        if (sources[i] && source_lens[i] > fec::kMaxPacketBufferSize)
            return report(fec::Error::text("source payload longer than a packet buffer"));
    bool st = false;
    const int rc = report(d->dec->SubmitPayloadRefs(block_id, smallest_ssid, largest_ssid, biggest, sources,
                                                     source_lens, repairs, repair_lens, &d->q, &st));
    if (staged) *staged = st ? 1 : 0;
    return rc;
}

void fec_go_decoder_drop(fec_go_decoder* d, uint64_t block_id) {
    if (d) d->blocks.erase(block_id);
}

int fec_go_decoder_flush(fec_go_decoder* d) { return d ? report(d->dec->Flush()) : FEC_ERR_INVALID_ARG; }

int fec_go_decoder_poll(fec_go_decoder* d, int wait, uint64_t* block_ids, uint32_t* lens, uint64_t* offsets,
                        uint8_t* out, size_t out_cap, size_t max_blocks, size_t* nblocks) {
    if (nblocks) *nblocks = 0;
    if (!d || (max_blocks && (!block_ids || !lens || !offsets || (out_cap && !out)))) return FEC_ERR_INVALID_ARG;
    fec::Error err = wait ? d->dec->Drain() : d->dec->Poll();
    if (err.ok() && !wait && d->dec->InFlight() == 0 && d->dec->Staged() > 0) err = d->dec->Flush();   // as the encoder
    if (!err.ok()) return report(err);
    // take the queue, hand out what fits from the front, put the rest back in order
    std::vector<fec::RecoveredQueue::Item> all;
    fec::RecoveredQueue::Item it;
    while (d->q.Pop(&it)) all.push_back(std::move(it));
    size_t n = 0, used = 0;
    for (; n < max_blocks && n < all.size() && used + all[n].payload.len <= out_cap; ++n) {
        block_ids[n] = all[n].block_id;
        lens[n] = (uint32_t)all[n].payload.len;
        offsets[n] = used;
        if (all[n].payload.len) memcpy(out + used, all[n].payload.data(), all[n].payload.len);
        used += all[n].payload.len;
    }
    const bool head_too_big = n == 0 && max_blocks && !all.empty();
    const size_t need = head_too_big ? all[0].payload.len : 0;
    for (size_t i = n; i < all.size(); ++i) d->q.Push(std::move(all[i]));
    if (head_too_big)   // the next payload alone exceeds out_cap: polling again would never progress
        return report(fec::Error{"recovered payload of " + std::to_string(need) + " bytes exceeds the poll buffer",
                                 FEC_ERR_INVALID_ARG});
    if (nblocks) *nblocks = n;
    return report(fec::Error::nil());
}

}  // extern "C"
