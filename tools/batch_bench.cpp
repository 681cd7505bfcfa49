// batch_bench.cpp — host-resident sender and receiver paths, per block vs batched (diagnostics).
//
// Feeds `conns` connections x `blocks` blocks of k source symbols (random bytes, `len`-byte
// payloads) through the C++ mirror of internal/fec:
//   per-block: Manager::AddSourceSymbolFrame -> repairSymbols -> one FEC_HOST encode per block
//              (the reference's call pattern, packet_packer.go:1005 -> manager.go:145)
//   batched:   Manager::AddSourceSymbolFrameBatched -> BatchEncoder (max_blocks per batch,
//              pinned staging, one H2D + launch + D2H per batch), frames into RepairQueues
// and the receiver the same way (HandleRepairFrame per block vs HandleRepairFrameBatched ->
// BatchDecoder), one lost source symbol per block; reports wall time, blocks/s and payload GB/s
// for each, checking the two produce the same frames and recovered payloads.
// Build: tools/batch_bench.sh.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <memory>
#include <random>
#include <vector>

#include "../include/fec_batch.hpp"

using namespace fec;

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
    const int k = argc > 1 ? atoi(argv[1]) : 20;
    const int m = argc > 2 ? atoi(argv[2]) : 10;
    const int conns = argc > 3 ? atoi(argv[3]) : 16;
    const int blocks = argc > 4 ? atoi(argv[4]) : 256;
    const size_t len = argc > 5 ? (size_t)atoi(argv[5]) : 1200;
    const size_t maxb = argc > 6 ? (size_t)atoi(argv[6]) : 1024;
    std::mt19937_64 rng(0x0FEC);
    std::vector<std::vector<uint8_t>> payloads((size_t)conns * blocks * k, std::vector<uint8_t>(len));
    for (auto& p : payloads)
        for (auto& b : p) b = (uint8_t)rng();
    auto engine = std::make_shared<Engine>(0);

    // per-block path
    std::vector<std::unique_ptr<Manager>> mgrs(conns);
    for (auto& mg : mgrs) {
        std::unique_ptr<ReedSolomonScheme> s;
        if (!ReedSolomonScheme::New(k, m, engine, &s).ok()) return 1;
        if (!Manager::New(std::move(s), k, m, &mg).ok()) return 1;
    }
    std::vector<std::vector<RepairFrame>> want(conns);
    {   // warm: context, code tables
        std::unique_ptr<ReedSolomonScheme> s;
        ReedSolomonScheme::New(k, m, engine, &s);
        std::unique_ptr<Manager> w;
        Manager::New(std::move(s), k, m, &w);
        std::vector<RepairFrame> out;
        for (int i = 0; i < k; ++i) w->AddSourceSymbolFrame(SourceSymbolFrame{(uint64_t)i, Slice::from(payloads[i].data(), len, kMaxPacketBufferSize)}, &out);
    }
    double t0 = now();
    for (int sym = 0; sym < blocks * k; ++sym)
        for (int c = 0; c < conns; ++c) {
            std::vector<RepairFrame> out;
            const auto& p = payloads[((size_t)c * blocks * k) + sym];
            Error e = mgrs[c]->AddSourceSymbolFrame(SourceSymbolFrame{(uint64_t)sym, Slice::from(p.data(), len, kMaxPacketBufferSize)}, &out);
            if (!e.ok()) { fprintf(stderr, "per-block: %s\n", e.msg.c_str()); return 1; }
            for (auto& f : out) want[c].push_back(f);
        }
    const double t_block = now() - t0;

    // batched path
    std::vector<std::unique_ptr<Manager>> bm(conns);
    for (auto& mg : bm) {
        std::unique_ptr<ReedSolomonScheme> s;
        ReedSolomonScheme::New(k, m, engine, &s);
        Manager::New(std::move(s), k, m, &mg);
    }
    std::unique_ptr<BatchEncoder> enc;
    if (!BatchEncoder::New(ReedSolomonFECScheme, k, m, maxb, std::make_shared<Engine>(0), &enc).ok()) return 1;
    std::vector<std::unique_ptr<RepairQueue>> qs(conns);
    for (auto& q : qs) q.reset(new RepairQueue(nullptr, (size_t)blocks * m));
    {   // warm: staging allocation, context
        std::unique_ptr<ReedSolomonScheme> s;
        ReedSolomonScheme::New(k, m, engine, &s);
        std::unique_ptr<Manager> w;
        Manager::New(std::move(s), k, m, &w);
        RepairQueue wq(nullptr, 1024);
        for (int i = 0; i < k; ++i) w->AddSourceSymbolFrameBatched(SourceSymbolFrame{(uint64_t)i, Slice::from(payloads[i].data(), len, kMaxPacketBufferSize)}, enc.get(), &wq);
        enc->Drain();
    }
    t0 = now();
    for (int sym = 0; sym < blocks * k; ++sym) {
        for (int c = 0; c < conns; ++c) {
            const auto& p = payloads[((size_t)c * blocks * k) + sym];
            Error e = bm[c]->AddSourceSymbolFrameBatched(SourceSymbolFrame{(uint64_t)sym, Slice::from(p.data(), len, kMaxPacketBufferSize)}, enc.get(), qs[c].get());
            if (!e.ok()) { fprintf(stderr, "batched: %s\n", e.msg.c_str()); return 1; }
        }
        if (sym % k == k - 1) enc->Poll();
    }
    Error e = enc->Drain();
    const double t_batch = now() - t0;
    if (!e.ok()) { fprintf(stderr, "drain: %s\n", e.msg.c_str()); return 1; }

    bool same = true;
    for (int c = 0; c < conns && same; ++c) {
        size_t i = 0;
        for (const RepairFrame* f; (f = qs[c]->Peek()); qs[c]->Pop(), ++i) {
            if (i >= want[c].size() || f->block_id != want[c][i].block_id || f->parity_id != want[c][i].parity_id ||
                f->payload.len != want[c][i].payload.len ||
                memcmp(f->payload.data(), want[c][i].payload.data(), f->payload.len)) {
                same = false;
                break;
            }
        }
        same = same && i == want[c].size();
    }
    // ---- receive side: every block loses source symbol (b % k); the repair frames arrive
    // after the surviving sources (HandleRepairFrame fires recovery on the first repair)
    std::vector<std::vector<std::pair<BlockID, std::vector<uint8_t>>>> rwant(conns);
    std::vector<std::unique_ptr<Manager>> rm(conns), rbm(conns);
    for (int c = 0; c < conns; ++c) {
        std::unique_ptr<ReedSolomonScheme> s1, s2;
        ReedSolomonScheme::New(k, m, engine, &s1);
        ReedSolomonScheme::New(k, m, engine, &s2);
        Manager::New(std::move(s1), k, m, &rm[c]);
        Manager::New(std::move(s2), k, m, &rbm[c]);
    }
    auto feed_sources = [&](std::vector<std::unique_ptr<Manager>>& ms, int blk) {
        for (int c = 0; c < conns; ++c)
            for (int j = 0; j < k; ++j) {
                if (j == blk % k) continue;
                const int sym = blk * k + j;
                const auto& p = payloads[((size_t)c * blocks * k) + sym];
                Slice out;
                ms[c]->HandleSourceSymbolFrame(SourceSymbolFrame{(uint64_t)sym, Slice::from(p.data(), len, kMaxPacketBufferSize)}, &out);
            }
    };
    t0 = now();
    for (int blk = 0; blk < blocks; ++blk) {
        feed_sources(rm, blk);
        for (int c = 0; c < conns; ++c) {
            const RepairFrame& f = want[c][(size_t)blk * m];
            Slice out;
            Error e2 = rm[c]->HandleRepairFrame(RepairFrame{f.block_id, f.parity_id, Slice::from(f.payload.data(), f.payload.len, f.payload.len)}, &out);
            if (!e2.ok()) { fprintf(stderr, "per-block recv: %s\n", e2.msg.c_str()); return 1; }
            if (!out.nil()) rwant[c].push_back({f.block_id, out.bytes()});
        }
    }
    const double t_rblock = now() - t0;
    std::unique_ptr<BatchDecoder> dec;
    if (!BatchDecoder::New(ReedSolomonFECScheme, k, m, maxb, std::make_shared<Engine>(0), &dec).ok()) return 1;
    std::vector<std::unique_ptr<RecoveredQueue>> rq(conns);
    for (auto& q : rq) q.reset(new RecoveredQueue());
    {   // warm: staging allocation, context
        std::unique_ptr<ReedSolomonScheme> s;
        ReedSolomonScheme::New(k, m, engine, &s);
        std::unique_ptr<Manager> w;
        Manager::New(std::move(s), k, m, &w);
        RecoveredQueue wq;
        Slice out;
        for (int j = 1; j < k; ++j)
            w->HandleSourceSymbolFrame(SourceSymbolFrame{(uint64_t)j, Slice::from(payloads[j].data(), len, kMaxPacketBufferSize)}, &out);
        const RepairFrame& f = want[0][0];
        w->HandleRepairFrameBatched(RepairFrame{f.block_id, f.parity_id, Slice::from(f.payload.data(), f.payload.len, f.payload.len)}, dec.get(), &wq);
        dec->Drain();
    }
    t0 = now();
    for (int blk = 0; blk < blocks; ++blk) {
        feed_sources(rbm, blk);
        for (int c = 0; c < conns; ++c) {
            const RepairFrame& f = want[c][(size_t)blk * m];
            Error e2 = rbm[c]->HandleRepairFrameBatched(RepairFrame{f.block_id, f.parity_id, Slice::from(f.payload.data(), f.payload.len, f.payload.len)}, dec.get(), rq[c].get());
            if (!e2.ok()) { fprintf(stderr, "batched recv: %s\n", e2.msg.c_str()); return 1; }
        }
        dec->Poll();
    }
    e = dec->Drain();
    const double t_rbatch = now() - t0;
    if (!e.ok()) { fprintf(stderr, "recv drain: %s\n", e.msg.c_str()); return 1; }
    bool rsame = true;
    for (int c = 0; c < conns && rsame; ++c) {
        RecoveredQueue::Item it;
        size_t i = 0;
        while (rq[c]->Pop(&it)) {
            if (i >= rwant[c].size() || it.block_id != rwant[c][i].first || it.payload.bytes() != rwant[c][i].second) {
                rsame = false;
                break;
            }
            ++i;
        }
        rsame = rsame && i == rwant[c].size();
    }

    const double nblk = (double)conns * blocks;
    const double bytes = nblk * k * len;
    printf("{\"k\": %d, \"m\": %d, \"connections\": %d, \"blocks\": %.0f, \"payload_bytes\": %zu, \"max_batch\": %zu, "
           "\"per_block_s\": %.4f, \"per_block_blocks_per_s\": %.0f, \"per_block_GB/s\": %.3f, "
           "\"batched_s\": %.4f, \"batched_blocks_per_s\": %.0f, \"batched_GB/s\": %.3f, \"speedup\": %.1f, "
           "\"frames_identical\": %s, \"recv_per_block_s\": %.4f, \"recv_per_block_blocks_per_s\": %.0f, "
           "\"recv_batched_s\": %.4f, \"recv_batched_blocks_per_s\": %.0f, \"recv_speedup\": %.1f, "
           "\"recovered_identical\": %s}\n",
           k, m, conns, nblk, len, maxb, t_block, nblk / t_block, bytes / t_block / 1e9, t_batch, nblk / t_batch,
           bytes / t_batch / 1e9, t_block / t_batch, same ? "true" : "false", t_rblock, nblk / t_rblock, t_rbatch,
           nblk / t_rbatch, t_rblock / t_rbatch, rsame ? "true" : "false");
    return same && rsame ? 0 : 2;
}
