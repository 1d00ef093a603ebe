// tests/native/engine_host_stub.cpp — TEST ONLY.
//
// Lets the product's HOST logic (tx parser, interpreter, deferring checker, sighash job builder,
// round/re-run stitching in csrc/host/*.cpp) run in a CPU-only test build: this file replaces
// the device pipeline (csrc/sighash.hip + ecdsa_verify.hip) with the ORACLE (oracle/bcc_oracle.c)
// evaluating the very jobs the host built (unpad -> SHA-256d -> patch -> SHA-256d -> ECDSA).
// It is linked only into tests/native/_build/engine_host.so, never into librbc_amd.so.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../oracle/bcc_oracle.h"
#include "../../rust-bitcoinconsensus_amd/csrc/pipeline.h"
#include "../../rust-bitcoinconsensus_amd/csrc/host/engine.h"
#include "../../rust-bitcoinconsensus_amd/csrc/host/host_verify.h"

namespace bcc {

static size_t unpadded_len(const uint8_t* m, size_t padded) {
    uint64_t bits = 0;
    for (int i = 0; i < 8; i++) bits = (bits << 8) | m[padded - 8 + i];
    return (size_t)(bits / 8);
}

static void stub_sighash(const SighashJobs& j, std::vector<uint8_t>& msg);
static void stub_ecdsa(const TupleRows& rows, const uint8_t* msg, uint8_t* verdict);
void set_stage_threads(unsigned) {}  // the device batch is stubbed out
static bool stub_direct = true;
void set_direct_upload(bool on) { stub_direct = on; }
bool direct_upload() { return stub_direct; }
void* pinned_alloc(size_t bytes) {  // ordinary memory: nothing is uploaded here
    void* p = malloc(bytes ? bytes : 1);
    if (!p) throw std::bad_alloc();
    return p;
}
void pinned_free(void* p, size_t) noexcept { free(p); }
void pinned_trim() {}
void release_device_thread_state() {}
void release_tuple_thread_state() {}
// Early Q halves: the stub keeps the calling thread's early rows and checks that every row the
// engine maps to an early twin (TupleRows::emap) is that twin byte for byte (tag, x, y, r, s) --
// the property DeviceBatch's K_keyq copy relies on; the verdicts are computed in full regardless.
thread_local TupleRows tl_early;
thread_local size_t tl_early_checked = 0, tl_early_msg_checked = 0;
static void stub_tpl_digest(const SighashJobs& j, const TplJob& t, uint8_t out[32]);
// Early sighashes: the early jobs' digests (oracle SHA-256d of the assembled preimages) land in
// tl_early.msg at their early rows; gpu_verify_parts compares every row that takes one (mmap) with
// the digest of its own job.
int gpu_early_launch(int, const TupleRows* const* rows, size_t P, const SighashJobs* const* jobs) {
    tl_early.clear();
    for (size_t p = 0; p < P; p++) {
        const size_t r0 = tl_early.tag.size();
        TupleRows r = *rows[p];
        r.materialize();
        tl_early.msg.resize(32 * (r0 + r.size()), 0);
        if (jobs && jobs[p])
            for (const TplJob& t : jobs[p]->tjobs) {
                if (t.row >= r.size()) abort();
                stub_tpl_digest(*jobs[p], t, &tl_early.msg[32 * (r0 + t.row)]);
            }
        tl_early.tag.insert(tl_early.tag.end(), r.tag.begin(), r.tag.end());
        tl_early.x.insert(tl_early.x.end(), r.x.begin(), r.x.end());
        tl_early.y.insert(tl_early.y.end(), r.y.begin(), r.y.end());
        tl_early.r.insert(tl_early.r.end(), r.r.begin(), r.r.end());
        tl_early.s.insert(tl_early.s.end(), r.s.begin(), r.s.end());
    }
    return 0;
}
void gpu_early_reset(int) { tl_early.clear(); }
static void check_early_twins(const TupleRows& rw) {  // rw materialized
    for (size_t k = 0; k < rw.emap.size() && k < rw.size(); k++) {
        const uint32_t e = rw.emap[k];
        if (e == TupleRows::NO_EARLY) continue;
        const bool same = e < tl_early.size() && rw.tag[k] == tl_early.tag[e] &&
                          memcmp(&rw.x[32 * k], &tl_early.x[32 * (size_t)e], 32) == 0 &&
                          (rw.tag[k] == 2 || rw.tag[k] == 3 ||
                           memcmp(&rw.y[32 * k], &tl_early.y[32 * (size_t)e], 32) == 0) &&
                          memcmp(&rw.r[32 * k], &tl_early.r[32 * (size_t)e], 32) == 0 &&
                          memcmp(&rw.s[32 * k], &tl_early.s[32 * (size_t)e], 32) == 0;
        if (!same) {
            fprintf(stderr, "engine_host_stub: row %zu mapped to early row %u differs\n", k, e);
            abort();
        }
        tl_early_checked++;
    }
}
extern "C" size_t stub_early_checked(void) { return tl_early_checked; }
extern "C" size_t stub_early_msg_checked(void) { return tl_early_msg_checked; }
static void check_early_msgs(const TupleRows& rw, const uint8_t* msg) {  // msg: the round's digests
    for (size_t k = 0; k < rw.mmap.size() && k < rw.size(); k++) {
        const uint32_t e = rw.mmap[k];
        if (e == TupleRows::NO_EARLY) continue;
        if ((size_t)e >= tl_early.size() || memcmp(&tl_early.msg[32 * (size_t)e], msg + 32 * k, 32) != 0) {
            fprintf(stderr, "engine_host_stub: row %zu's early sighash (early row %u) differs\n", k, e);
            abort();
        }
        tl_early_msg_checked++;
    }
}
// As DeviceBatch: the rows are copied (staged) first, the sighash jobs hash into the copy, then the
// late rows (host-hashed while the device runs) land in it (put_late), then the ECDSA stage.
int gpu_verify_parts(int, const SighashJobs* const* jobs, const TupleRows* const* rows, size_t parts,
                     uint8_t* verdict, double*, const LateMsgFill* late) {
    std::vector<TupleRows> staged(parts);
    std::vector<uint8_t> msg;
    for (size_t p = 0; p < parts; p++) {
        staged[p] = *rows[p];
        staged[p].materialize();  // rows stored without y / msg (TupleRows::add_lazy): zero / ONE
        check_early_twins(staged[p]);
        std::vector<uint8_t> m = staged[p].msg;
        stub_sighash(*jobs[p], m);
        msg.insert(msg.end(), m.begin(), m.end());
    }
    if (late) {
        std::vector<uint32_t> lr;
        std::vector<uint8_t> ld;
        (*late)(lr, ld);
        if (ld.size() != 32 * lr.size()) return 1;
        for (size_t k = 0; k < lr.size(); k++) {
            if (32 * (size_t)lr[k] >= msg.size()) return 1;
            memcpy(&msg[32 * (size_t)lr[k]], &ld[32 * k], 32);
        }
    }
    size_t r0 = 0;
    for (size_t p = 0; p < parts; p++) {
        check_early_msgs(staged[p], &msg[32 * r0]);
        stub_ecdsa(staged[p], &msg[32 * r0], verdict + r0);
        r0 += staged[p].size();
    }
    return 0;
}

// The staged round: the parts are kept and evaluated when it runs (like the device's upload).
struct StagedRound {
    int dev;
    std::vector<const SighashJobs*> jobs;
    std::vector<const TupleRows*> rows;
    std::vector<uint8_t> verdicts;  // gpu_staged_launch's
    bool der = false;               // staged by gpu_staged_stage_der (verdicts already computed)
};
StagedRound* gpu_staged_new(int device) { return new StagedRound{device, {}, {}, {}, false}; }
void gpu_staged_free(StagedRound* s) { delete s; }
int gpu_staged_stage(StagedRound* s, const SighashJobs* const* jobs, const TupleRows* const* rows,
                     size_t parts, double*) {
    s->jobs.assign(jobs, jobs + parts);
    s->rows.assign(rows, rows + parts);
    s->der = false;
    return 0;
}
int gpu_staged_run(StagedRound* s, uint8_t* verdict, const LateMsgFill* late) {
    return gpu_verify_parts(s->dev, s->jobs.data(), s->rows.data(), s->jobs.size(), verdict,
                            nullptr, late);
}
// launch evaluates at once (the caller may rebuild its rows afterwards), finish copies
int gpu_staged_launch(StagedRound* s, const LateMsgFill* late) {
    if (s->der) return 0;
    size_t n = 0;
    for (const TupleRows* r : s->rows) n += r->size();
    std::vector<uint8_t>& v = s->verdicts;
    v.assign(n, 0);
    return gpu_staged_run(s, v.data(), late);
}
// per-shard row pre-upload: nothing to send here (the staged round evaluates its parts itself)
int gpu_staged_pre_arm(StagedRound*, unsigned, size_t) { return 0; }
void gpu_staged_pre_upload(StagedRound*, unsigned, const TupleRows&) {}
int gpu_staged_finish(StagedRound* s, uint8_t* verdict) {
    if (!s->verdicts.empty()) memcpy(verdict, s->verdicts.data(), s->verdicts.size());
    return 0;
}

// Raw tuples (bcc_pubkey_verify_batch, K_der on the device): the oracle's own CPubKey::Verify per
// tuple, from the caller's blobs -- so the CPU suite checks the entry point's slicing and offsets
// against the oracle, not the product's host parse against itself.
static void stub_der(const DerTuples& t, uint8_t* verdict) {
    const uint64_t pl = t.pub_off[0], ph = t.pub_off[t.n], sl = t.sig_off[0], sh = t.sig_off[t.n];
    for (size_t i = 0; i < t.n; i++) {
        const uint64_t p0 = t.pub_off[i], p1 = t.pub_off[i + 1], s0 = t.sig_off[i], s1 = t.sig_off[i + 1];
        verdict[i] = (pl <= p0 && p0 <= p1 && p1 <= ph && sl <= s0 && s0 <= s1 && s1 <= sh)
                         ? (uint8_t)bcco_pubkey_verify(t.pub_blob + p0, p1 - p0, t.msg32 + 32 * i,
                                                       t.sig_blob + s0, s1 - s0)
                         : 0;
    }
}
int gpu_verify_der(int, const DerTuples& t, uint8_t* verdict) {
    stub_der(t, verdict);
    return 0;
}
int gpu_staged_stage_der(StagedRound* s, const DerTuples& t, double*) {
    s->jobs.clear();
    s->rows.clear();
    s->verdicts.assign(t.n, 0);  // evaluated now (the caller's buffers outlive the round anyway)
    stub_der(t, s->verdicts.data());
    s->der = true;
    return 0;
}

// The sighash stage: msg rows (entering as rows.msg) overwritten by every job's digest.
static void stub_sighash(const SighashJobs& j, std::vector<uint8_t>& msg) {
    std::vector<uint8_t> auxd(32 * j.aux_off.size());
    for (size_t a = 0; a < j.aux_off.size(); a++) {
        const uint8_t* m = &j.aux[(size_t)j.aux_off[a] * 64];
        size_t L = (size_t)j.aux_nblk[a] * 64;
        bcco_sha256d(m, unpadded_len(m, L), &auxd[32 * a]);
    }
    std::vector<uint8_t> pre(j.pre.begin(), j.pre.end());
    for (const auto& p : j.patches) memcpy(&pre[p.pre_byte], &auxd[32 * p.aux], 32);
    for (size_t k = 0; k < j.pre_off.size(); k++) {
        const uint8_t* m = &pre[(size_t)j.pre_off[k] * 64];
        size_t L = (size_t)j.pre_nblk[k] * 64;
        bcco_sha256d(m, unpadded_len(m, L), &msg[32 * j.pre_row[k]]);
    }
    for (const TplJob& t : j.tjobs) {  // template jobs: assemble the preimage, then hash
        stub_tpl_digest(j, t, &msg[32 * t.row]);
        if (tpl_has_mid(t)) {  // the product's midstate path must give the same digest
            uint8_t d[32];
            host::tpl_job_sighash(j.tpl.data(), j.code.data(), t, d);
            if (memcmp(d, &msg[32 * t.row], 32) != 0) {
                fprintf(stderr, "engine_host_stub: template midstate digest mismatch (row %u)\n", t.row);
                abort();
            }
        }
    }
    for (const WinJob& w : j.wjobs) {  // BIP143 from the raw tx: the oracle's own sighash
        const WtxRec& r = j.wtx[w.tx];
        const uint8_t* c = &j.code[w.code_off];
        size_t hdr = c[0] < 253 ? 1 : c[0] == 253 ? 3 : 5;
        const int64_t amount = (int64_t)((uint64_t)w.amount_hi << 32 | w.amount_lo);
        bcco_sighash(&j.txraw[r.tx_off], r.tx_len, w.nin, c + hdr, w.code_len - hdr,
                     (int)w.hashtype, amount, 1, &msg[32 * w.row]);
    }
}

// A legacy template job's digest from its full preimage (template | code field | template rest |
// hashtype), whatever its flags (TPL_MID / TPL_EARLY only change how the device gets there).
static void stub_tpl_digest(const SighashJobs& j, const TplJob& t, uint8_t out[32]) {
    std::vector<uint8_t> m(j.tpl.begin() + t.tpl_off, j.tpl.begin() + t.tpl_off + t.pos);
    m.insert(m.end(), j.code.begin() + t.code_off, j.code.begin() + t.code_off + t.code_len);
    m.insert(m.end(), j.tpl.begin() + t.tpl_off + t.pos + 1, j.tpl.begin() + t.tpl_off + t.tpl_len);
    for (int b = 0; b < 4; b++) m.push_back((uint8_t)(t.hashtype >> (8 * b)));
    bcco_sha256d(m.data(), m.size(), out);
}

int gpu_verify_batch(int dev, const SighashJobs& j, const TupleRows& rows, uint8_t* verdict, double*) {
    const SighashJobs* jp = &j;
    const TupleRows* rp = &rows;
    return gpu_verify_parts(dev, &jp, &rp, 1, verdict, nullptr, nullptr);
}

static void stub_ecdsa(const TupleRows& rows, const uint8_t* msg, uint8_t* verdict) {
    for (size_t i = 0; i < rows.size(); i++) {
        uint8_t pub[65];
        pub[0] = rows.tag[i];
        memcpy(pub + 1, &rows.x[32 * i], 32);
        memcpy(pub + 33, &rows.y[32 * i], 32);
        size_t plen = (pub[0] == 2 || pub[0] == 3) ? 33 : 65;
        uint8_t qx[32], qy[32];
        if (!bcco_pubkey_parse(pub, plen, qx, qy)) {
            verdict[i] = 0;
            continue;
        }
        verdict[i] = (uint8_t)bcco_ecdsa_verify_raw(qx, qy, &rows.r[32 * i], &rows.s[32 * i],
                                                    &msg[32 * i]);
    }
    bcc::host::apply_key_hashes(rows, verdict);  // the device's key_hash_kernel
}

// BIP341 jobs (host/taproot.cpp): aux messages single SHA-256, patch, TapSighash over the
// tag prefix + the message (the length field of a message counts the 64-byte tag block), BIP340.
int gpu_taproot_verify(int, const TaprootJobs& j, uint8_t* verdict, uint8_t* msg32_out);
int gpu_taproot_verify_parts(int dev, const TaprootJobs* const* parts, size_t P, uint8_t* verdict,
                             uint8_t* msg32_out) {
    size_t r0 = 0;
    for (size_t q = 0; q < P; q++) {
        gpu_taproot_verify(dev, *parts[q], verdict + r0, msg32_out ? msg32_out + 32 * r0 : nullptr);
        r0 += parts[q]->rows();
    }
    return 0;
}

// The two-phase form: begin evaluates at once (the parts are rebuilt after it returns), end copies.
static thread_local std::vector<uint8_t> tl_tap_verdict[2], tl_tap_msg[2];
int gpu_taproot_begin(int dev, int slot, const TaprootJobs* const* parts, size_t P) {
    size_t n = 0;
    for (size_t q = 0; q < P; q++) n += parts[q]->rows();
    tl_tap_verdict[slot].assign(n, 0);
    tl_tap_msg[slot].assign(32 * n, 0);
    return gpu_taproot_verify_parts(dev, parts, P, tl_tap_verdict[slot].data(), tl_tap_msg[slot].data());
}
int gpu_taproot_end(int, int slot, uint8_t* verdict, uint8_t* msg32_out) {
    const size_t n = tl_tap_verdict[slot].size();
    if (n) memcpy(verdict, tl_tap_verdict[slot].data(), n);
    if (msg32_out && n) memcpy(msg32_out, tl_tap_msg[slot].data(), 32 * n);
    tl_tap_verdict[slot].clear();
    return 0;
}

int gpu_taproot_verify(int, const TaprootJobs& j, uint8_t* verdict, uint8_t* msg32_out) {
    std::vector<uint8_t> auxd(32 * j.aux_off.size());
    for (size_t a = 0; a < j.aux_off.size(); a++) {
        const uint8_t* m = &j.aux[(size_t)j.aux_off[a] * 64];
        bcco_sha256(m, unpadded_len(m, (size_t)j.aux_nblk[a] * 64), &auxd[32 * a]);
    }
    std::vector<uint8_t> msgs(j.msg.begin(), j.msg.end());
    for (const auto& p : j.patches) memcpy(&msgs[p.pre_byte], &auxd[32 * p.aux], 32);
    uint8_t tag[32];
    bcco_sha256(reinterpret_cast<const uint8_t*>("TapSighash"), 10, tag);
    const size_t n = j.rows();
    std::vector<uint8_t> h(32 * n, 0);
    bcc::host::taproot_dev_sigmsg_host(j.dev, h.data());  // the device-built SigMsg path
    for (size_t k = 0; k < j.msg_off.size(); k++) {
        const uint8_t* m = &msgs[(size_t)j.msg_off[k] * 64];
        size_t L = unpadded_len(m, (size_t)j.msg_nblk[k] * 64) - 64;
        std::vector<uint8_t> full(tag, tag + 32);
        full.insert(full.end(), tag, tag + 32);
        full.insert(full.end(), m, m + L);
        bcco_sha256(full.data(), full.size(), &h[32 * j.msg_row[k]]);
    }
    for (size_t i = 0; i < n; i++)
        verdict[i] = (uint8_t)bcco_schnorr_verify(&j.sig64[64 * i], &h[32 * i], &j.pk32[32 * i]);
    if (msg32_out) memcpy(msg32_out, h.data(), 32 * n);
    return 0;
}

}  // namespace bcc

// bcc_debug_sighash's host half (the job builder) with the stub sighash stage: the CPU suite
// checks the jobs the engine builds for the reference's sighash goldens.
extern "C" int stub_debug_sighash(const bcc::host::SighashCheck* c, size_t n, uint8_t* out) {
    bcc::SighashJobs jobs;
    bcc::TupleRows rows;
    if (bcc::host::build_sighash_checks(c, n, jobs, rows) != n) return -1;
    std::vector<uint8_t> msg = rows.msg;
    bcc::stub_sighash(jobs, msg);
    memcpy(out, msg.data(), msg.size());
    return 0;
}
