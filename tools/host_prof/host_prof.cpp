// Dev tool: profile the HOST half of bitcoinconsensus_verify_batch (deserialize, pre-checks,
// interpreter, sighash job building) on N synthetic P2WPKH spends, with the device pipeline
// replaced by a stub that answers "valid" for every deferred check.  Not part of the library.
//   g++ -O2 -pg ... (see tools/host_prof/run.sh)
#include <chrono>
#include <ctime>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/bitcoinconsensus.h"
#include "../../include/bcc_amd.h"
#include "../../rust-bitcoinconsensus_amd/csrc/host/hashes.h"
#include "../../rust-bitcoinconsensus_amd/csrc/pipeline.h"

namespace bcc {
int gpu_verify_batch(int, const SighashJobs&, const TupleRows& rows, uint8_t* verdict, double*) {
    memset(verdict, 1, rows.size());
    return 0;
}
void set_stage_threads(unsigned) {}  // the device batch is stubbed out
void set_direct_upload(bool) {}
bool direct_upload() { return true; }
void* pinned_alloc(size_t bytes) {  // ordinary memory: nothing is uploaded here
    void* p = malloc(bytes ? bytes : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void pinned_free(void* p, size_t) noexcept { free(p); }
void pinned_trim() {}
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
    memset(verdict, 1, n);
    return 0;
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
int gpu_early_launch(int, const TupleRows* const*, size_t, const SighashJobs* const*) { return 0; }  // early Q: no-op
void gpu_early_reset(int) {}
int gpu_verify_der(int, const DerTuples& t, uint8_t* verdict) {
    memset(verdict, 1, t.n);
    return 0;
}
int gpu_staged_stage_der(StagedRound* s, const DerTuples&, double*) {
    s->rows.clear();
    return 0;
}
// per-shard row pre-upload: nothing to send here (the staged round evaluates its parts itself)
int gpu_staged_pre_arm(StagedRound*, unsigned, size_t) { return 0; }
void gpu_staged_pre_upload(StagedRound*, unsigned, const TupleRows&) {}
int gpu_staged_finish(StagedRound* s, uint8_t* verdict) {
    return gpu_staged_run(s, verdict, nullptr);
}
namespace host {
void taproot_release_thread_state() {}  // taproot.cpp is not linked here
}  // namespace host
}  // namespace bcc

static void le(std::vector<uint8_t>& o, uint64_t v, int k) {
    for (int i = 0; i < k; i++) o.push_back((uint8_t)(v >> (8 * i)));
}

int main(int argc, char** argv) {
    size_t n = argc > 1 ? (size_t)atol(argv[1]) : 200000;
    std::vector<std::vector<uint8_t>> txs(n), spks(n);
    for (size_t i = 0; i < n; i++) {
        uint8_t pub[33], h[20], sig[72];
        pub[0] = 2;
        for (int k = 1; k < 33; k++) pub[k] = (uint8_t)(i * 131 + k * 7);
        bcc::host::hash160(pub, 33, h);
        spks[i] = {0x00, 0x14};
        spks[i].insert(spks[i].end(), h, h + 20);
        // strict-DER (r, s) of 32 bytes each, + SIGHASH_ALL
        sig[0] = 0x30; sig[1] = 68; sig[2] = 0x02; sig[3] = 32;
        for (int k = 0; k < 32; k++) sig[4 + k] = (uint8_t)(0x11 + i + k);
        sig[4] &= 0x7f;
        sig[36] = 0x02; sig[37] = 32;
        for (int k = 0; k < 32; k++) sig[38 + k] = (uint8_t)(0x22 + i * 3 + k);
        sig[38] &= 0x7f;
        sig[70] = 0x01;
        auto& t = txs[i];
        le(t, 2, 4);
        t.push_back(0); t.push_back(1);
        t.push_back(1);
        for (int k = 0; k < 32; k++) t.push_back((uint8_t)(i >> (k % 8)));
        le(t, 0, 4);
        t.push_back(0);
        le(t, 0xffffffffu, 4);
        t.push_back(1);
        le(t, 1000 + i, 8);
        t.push_back(22); t.push_back(0); t.push_back(0x14);
        for (int k = 0; k < 20; k++) t.push_back((uint8_t)k);
        t.push_back(2);
        t.push_back(71);
        t.insert(t.end(), sig, sig + 71);
        t.push_back(33);
        t.insert(t.end(), pub, pub + 33);
        le(t, 0, 4);
    }
    std::vector<bcc_batch_item> items(n);
    for (size_t i = 0; i < n; i++)
        items[i] = bcc_batch_item{spks[i].data(), (unsigned)spks[i].size(), (int64_t)(5000 + i),
                                  txs[i].data(), (unsigned)txs[i].size(), 0};
    std::vector<int> ret(n);
    std::vector<bitcoinconsensus_error> err(n);
    for (int rep = 0; rep < 3; rep++) {
        timespec c0, c1;
        clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c0);
        auto t0 = std::chrono::steady_clock::now();
        long v = bitcoinconsensus_verify_batch(items.data(), n, 0xE15, ret.data(), err.data());
        double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &c1);
        const double cpu_ms = 1e3 * (c1.tv_sec - c0.tv_sec) + 1e-6 * (c1.tv_nsec - c0.tv_nsec);
        bcc_batch_stats st;
        bcc_last_batch_stats(&st);
        printf("cpu %.1f ms | n %zu valid %ld  %.1f ms  %.2f M items/s | prepare %.1f interpret %.1f merge %.1f "
               "stage %.1f gpu %.1f host %.1f total %.1f ms | key hashes on the device %zu\n", cpu_ms, n, v, 1e3 * s, n / s / 1e6,
               1e3 * st.prepare_seconds, 1e3 * st.interpret_seconds, 1e3 * st.merge_seconds,
               1e3 * st.stage_seconds, 1e3 * st.gpu_seconds, 1e3 * st.host_seconds,
               1e3 * st.total_seconds, st.device_key_hashes);
        printf("    prepare lag %.2f parse(max) %.2f hash %.2f | interpret shard max %.2f mean %.2f | "
               "stitch %.2f finish %.2f ms | process cpu %.1f ms\n",
               1e3 * st.prepare_lag_seconds, 1e3 * st.prepare_parse_seconds, 1e3 * st.prepare_hash_seconds,
               1e3 * st.interpret_shard_max_seconds, 1e3 * st.interpret_shard_mean_seconds,
               1e3 * st.stitch_seconds, 1e3 * st.finish_seconds, 1e3 * st.process_cpu_seconds);
    }
    return 0;
}
