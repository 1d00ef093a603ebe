// tools/pipe_probe — CPU-only probe of bitcoinconsensus_verify_batch's pipelining (VERDICT r03
// item 3): the product's host engine (csrc/host/*.cpp, unchanged) with the device round replaced
// by a SLEEP of `ns_per_tuple` x tuples on the calling worker (every verdict 1), over N synthetic
// P2WPKH spends with well-formed but unsigned signatures.  Pipelined (chunk > 0) and unpipelined
// calls are timed with the engine's own bcc_batch_stats, so chunking overhead and interference from
// the device thread can be told apart without a GPU.  Not part of the product or the tests.
//
//   tools/pipe_probe/build.sh && tools/pipe_probe/pipe_probe N NS_PER_TUPLE CALLS CHUNK [CHUNK...]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../rust-bitcoinconsensus_amd/csrc/pipeline.h"
#include "../../rust-bitcoinconsensus_amd/csrc/host/engine.h"
#include "../../rust-bitcoinconsensus_amd/csrc/host/hashes.h"
#include "bcc_amd.h"
#include "bitcoinconsensus.h"

static double g_ns_per_tuple = 21.0;

namespace bcc {
void set_stage_threads(unsigned) {}
void release_device_thread_state() {}
void release_tuple_thread_state() {}
int gpu_verify_parts(int, const SighashJobs* const*, const TupleRows* const* rows, size_t parts,
                     uint8_t* verdict, double*, const LateMsgFill* late) {
    if (late) {
        std::vector<uint32_t> lr;
        std::vector<uint8_t> ld;
        (*late)(lr, ld);
    }
    size_t n = 0;
    for (size_t p = 0; p < parts; p++) n += rows[p]->size();
    std::this_thread::sleep_for(std::chrono::nanoseconds((long long)(g_ns_per_tuple * n)));
    memset(verdict, 1, n);
    return 0;
}
int gpu_verify_batch(int d, const SighashJobs& j, const TupleRows& r, uint8_t* v, double* s) {
    const SighashJobs* jp = &j;
    const TupleRows* rp = &r;
    return gpu_verify_parts(d, &jp, &rp, 1, v, s);
}
struct StagedRound {
    std::vector<const TupleRows*> rows;
};
StagedRound* gpu_staged_new(int) { return new StagedRound{}; }
void gpu_staged_free(StagedRound* s) { delete s; }
int gpu_staged_stage(StagedRound* s, const SighashJobs* const*, const TupleRows* const* rows,
                     size_t parts, double*) {
    s->rows.assign(rows, rows + parts);
    return 0;
}
int gpu_staged_run(StagedRound* s, uint8_t* verdict, const LateMsgFill* late) {
    return gpu_verify_parts(0, nullptr, s->rows.data(), s->rows.size(), verdict, nullptr, late);
}
int gpu_staged_launch(StagedRound*, const LateMsgFill*) { return 0; }
int gpu_staged_finish(StagedRound* s, uint8_t* verdict) {
    return gpu_staged_run(s, verdict, nullptr);
}
int gpu_taproot_verify_parts(int, const TaprootJobs* const*, size_t, uint8_t*, uint8_t*) { return -1; }
}  // namespace bcc

struct Spend {
    std::vector<uint8_t> tx, spk;
};

static Spend make_spend(std::mt19937_64& rng) {
    auto rnd = [&](uint8_t* p, size_t n) {
        for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rng();
    };
    uint8_t pub[33];
    pub[0] = 2 + (rng() & 1);
    rnd(pub + 1, 32);
    uint8_t h[20];
    bcc::host::hash160(pub, 33, h);
    Spend s;
    s.spk = {0x00, 0x14};
    s.spk.insert(s.spk.end(), h, h + 20);
    uint8_t r[32], ss[32];
    rnd(r, 32);
    rnd(ss, 32);
    r[0] = (r[0] & 0x7f) | 0x01;  // 32-byte positive r
    ss[0] = (ss[0] & 0x3f) | 0x01;  // low S
    std::vector<uint8_t> sig = {0x30, 0x44, 0x02, 0x20};
    sig.insert(sig.end(), r, r + 32);
    sig.push_back(0x02);
    sig.push_back(0x20);
    sig.insert(sig.end(), ss, ss + 32);
    sig.push_back(0x01);  // SIGHASH_ALL
    auto& t = s.tx;
    auto le32 = [&](uint32_t v) {
        for (int i = 0; i < 4; i++) t.push_back((uint8_t)(v >> (8 * i)));
    };
    le32(2);
    t.push_back(0);
    t.push_back(1);  // marker, flag
    t.push_back(1);  // one input
    uint8_t prev[36];
    rnd(prev, 36);
    t.insert(t.end(), prev, prev + 36);
    t.push_back(0);  // empty scriptSig
    le32(0xfffffffe);
    t.push_back(1);  // one output
    for (int i = 0; i < 8; i++) t.push_back(i == 1 ? 0x10 : 0);
    t.push_back(22);
    t.insert(t.end(), s.spk.begin(), s.spk.end());
    t.push_back(2);  // witness: sig, pubkey
    t.push_back((uint8_t)sig.size());
    t.insert(t.end(), sig.begin(), sig.end());
    t.push_back(33);
    t.insert(t.end(), pub, pub + 33);
    le32(0);
    return s;
}

int main(int argc, char** argv) {
    const size_t N = argc > 1 ? (size_t)atoll(argv[1]) : 1000000;
    g_ns_per_tuple = argc > 2 ? atof(argv[2]) : 21.0;
    const int calls = argc > 3 ? atoi(argv[3]) : 5;
    std::vector<size_t> chunks;
    for (int i = 4; i < argc; i++) chunks.push_back((size_t)atoll(argv[i]));
    if (chunks.empty()) chunks = {0, 262144};
    std::mt19937_64 rng(7);
    std::vector<Spend> sp(N);
    for (auto& s : sp) s = make_spend(rng);
    std::vector<bcc_batch_item> items(N);
    for (size_t i = 0; i < N; i++)
        items[i] = bcc_batch_item{sp[i].spk.data(), (unsigned)sp[i].spk.size(), 4096,
                                  sp[i].tx.data(), (unsigned)sp[i].tx.size(), 0};
    std::vector<int> ret(N);
    printf("N %zu ns_per_tuple %.1f host_threads %u cpu_share %u\n", N, g_ns_per_tuple,
           bcc_get_host_threads(), bcc_cpu_share());
    for (size_t ch : chunks) {
        bcc_set_pipeline_chunk(ch);
        for (int c = 0; c < calls; c++) {
            auto t0 = std::chrono::steady_clock::now();
            long v = bitcoinconsensus_verify_batch(items.data(), N, 0xE15, ret.data(), nullptr);
            double ms = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() * 1e3;
            bcc_batch_stats st;
            bcc_last_batch_stats(&st);
            printf("chunk %7zu call %d valid %ld total %7.2f ms  prepare %6.2f (lag %5.2f parse %6.2f "
                   "hash %5.2f) interpret %6.2f stitch %5.2f finish %5.2f gpu_wait %6.2f  %.2f M/s\n",
                   ch, c, v, ms, st.prepare_seconds * 1e3, st.prepare_lag_seconds * 1e3,
                   st.prepare_parse_seconds * 1e3, st.prepare_hash_seconds * 1e3,
                   st.interpret_seconds * 1e3, st.stitch_seconds * 1e3, st.finish_seconds * 1e3,
                   st.gpu_seconds * 1e3, N / ms / 1e3);
        }
    }
    return 0;
}
