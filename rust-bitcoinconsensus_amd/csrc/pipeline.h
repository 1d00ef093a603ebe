// Internal (C++) interface of the device pipeline: host-built signature jobs -> HBM ->
//   K1 sha256d(aux messages)        BIP143 hashPrevouts / hashSequence / hashOutputs per tx
//   K2 patch(aux digests -> preimages)
//   K3 sha256d(preimages)           legacy + BIP143 sighashes, written as the tuple msg rows
//   K3' sha256d(template jobs)      legacy SIGHASH_ALL sighashes assembled from per-tx templates
//   K4 ecdsa_verify(tuples)         csrc/ecdsa_verify.hip
// All four launch back-to-back on one stream with inputs resident in HBM.
#pragma once
#include <cstddef>
#include <cstdint>
#include <algorithm>
#include <cstring>
#include <vector>
#include <functional>

namespace bcc {

// Page-locked host memory for the arrays a device round uploads as they are (round 6): the
// interpreter writes the tuple rows, the raw txs and the sighash blobs straight into buffers the
// DMA engine reads, so staging copies only the records whose offsets it rebases
// (DeviceBatch::stage_parts).  Blocks come from a process-wide pool in power-of-two classes and go
// back to it, never to the runtime while the process runs (a hipHostFree would wait for the GPU in
// the middle of a host pass), except through pinned_trim().  Without a device the pool hands out
// ordinary memory (sighash.hip; the CPU test build's stub uses malloc).
void* pinned_alloc(size_t bytes);
void pinned_free(void* p, size_t bytes) noexcept;
void pinned_trim();
template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U>&) {}
    T* allocate(size_t n) { return static_cast<T*>(pinned_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t n) noexcept { pinned_free(p, n * sizeof(T)); }
    template <class U>
    bool operator==(const PinnedAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U>&) const { return false; }
};
template <class T>
using pinned_vector = std::vector<T, PinnedAlloc<T>>;
using pinned_bytes = pinned_vector<uint8_t>;

struct PatchRec {
    uint32_t pre_byte;  // absolute byte offset in the padded preimage buffer
    uint32_t aux;       // index of the aux message whose digest goes there
};

// SHA-256 padding appended on the host so that the kernels only run whole 64-byte blocks.
// `prefix` = bytes already absorbed into the starting midstate (a tagged hash's 64-byte tag
// block): they count in the length field but are not part of m.
inline size_t sha_padded_len(size_t n) { return ((n + 8) / 64 + 1) * 64; }
template <class Buf>
inline void sha_append_padded(Buf& buf, const uint8_t* m, size_t n, size_t prefix = 0) {
    size_t L = sha_padded_len(n), base = buf.size();
    buf.resize(base + L, 0);
    if (n) memcpy(&buf[base], m, n);
    buf[base + n] = 0x80;
    uint64_t bits = (uint64_t)(n + prefix) * 8;
    for (int i = 0; i < 8; i++) buf[base + L - 1 - i] = (uint8_t)(bits >> (8 * i));
}

// A legacy SIGHASH_ALL job (interpreter.cpp:1273-1364) built on the device from its tx's
// template instead of a host preimage: message = T[0, pos) || code || T[pos + 1, tpl_len) ||
// le32(hashtype), where T is the tx serialized with every scriptSig empty (the byte at pos is the
// signing input's empty-script length byte) and code = compactsize || scriptCode without
// OP_CODESEPARATORs.  A tx's template is uploaded once per round; the O(nIn^2) preimage bytes of
// a many-input tx never exist on the host.
struct TplJob {
    uint32_t tpl_off;   // byte offset of T in the template blob (4-aligned)
    uint32_t tpl_len;
    uint32_t pos;
    uint32_t code_off;  // byte offset of code in the code blob (4-aligned)
    uint32_t code_len;
    uint32_t hashtype;  // serialized as le32 (a script's is the signature's last byte; the
                        // sighash goldens use any 32-bit value)
    uint32_t row;       // tuple row whose msg receives the sighash
    uint32_t nblk;      // padded message length in 64-byte blocks | TPL_MID when T carries midstates
};

// Round 5: the template midstates.  Every legacy preimage of a tx begins with T's first
// floor(pos / 64) blocks, so a long template is stored with the SHA-256 state after each of its
// whole blocks (mid[j]: j blocks absorbed, mid[0] = the IV; 8 native-order words each) right
// behind it, and a job flagged TPL_MID (in nblk) starts from mid[pos / 64] at block pos / 64: it hashes
// only the blocks from its splice on (a 442-input tx: 284 -> 1..284 blocks, half on average),
// on the device (K3') and on the host (hash_host_jobs) alike.
#if defined(__HIPCC__)
#define BCC_PL_HD __host__ __device__
#else
#define BCC_PL_HD
#endif
constexpr uint32_t TPL_MID = 0x80000000u;
constexpr uint32_t TPL_MID_MIN_BLOCKS = 8;  // shorter templates start from the IV
// Round 5, early sighashes: a job flagged TPL_EARLY (in nblk) has the same digest already computed
// in the call's early set (DeviceBatch::early_launch; its row's TupleRows::mmap names the early
// row), so the device's front lane skips it and the round copies that digest into the row instead.
// The host (fallback, small rounds) hashes it like any job; staging clears the flag when the early
// digests are not live for the round.
constexpr uint32_t TPL_EARLY = 0x40000000u;
BCC_PL_HD inline uint32_t tpl_mid_count(uint32_t tpl_len) { return (tpl_len - 1) / 64 + 1; }
BCC_PL_HD inline uint32_t tpl_mid_offset(uint32_t tpl_off, uint32_t tpl_len) {  // 4-aligned, after the 8 zero bytes
    return tpl_off + ((tpl_len + 3) & ~3u) + 8;
}
BCC_PL_HD inline uint32_t tpl_nblk(const TplJob& j) { return j.nblk & ~(TPL_MID | TPL_EARLY); }
BCC_PL_HD inline bool tpl_early(const TplJob& j) { return (j.nblk & TPL_EARLY) != 0; }
BCC_PL_HD inline bool tpl_has_mid(const TplJob& j) { return (j.nblk & TPL_MID) != 0; }
// The blocks a job hashes (from its start block: pos / 64 with midstates, else 0).
BCC_PL_HD inline uint32_t tpl_job_blocks(const TplJob& j) {
    return tpl_has_mid(j) ? tpl_nblk(j) - j.pos / 64 : tpl_nblk(j);
}
// Appends T (4-aligned, + 8 zero bytes) and, when mid != nullptr, its tpl_mid_count(n) midstates
// (8 words each) to a template blob; returns T's offset.
template <class Buf>
inline uint32_t append_tpl(Buf& blob, const uint8_t* m, size_t n,
                           const uint32_t* mid) {
    const uint32_t off = (uint32_t)blob.size();
    blob.insert(blob.end(), m, m + n);
    blob.resize(off + ((n + 3) & ~(size_t)3) + 8, 0);
    if (mid) {
        const size_t bytes = 32 * (size_t)tpl_mid_count((uint32_t)n);
        const size_t at = blob.size();
        blob.resize(at + bytes);
        memcpy(&blob[at], mid, bytes);
    }
    return off;
}

// BIP143 jobs built on the device from the raw transaction bytes: per tx a
// WtxRec (K_wtx parses the wire format, primitives/transaction.h:188-224 / serialize.h:318-347,
// records every input's outpoint / nSequence offsets and hashes hashPrevouts / hashSequence /
// hashOutputs, interpreter.cpp:1366-1397), per check a WinJob (K_win assembles the BIP143
// preimage, interpreter.cpp:1581-1625, from the tx bytes, those hashes and its own fields and
// hashes it into the tuple's msg row).  The host only appends the tx bytes once per round and a
// 40-byte record per check; no preimage or aux message exists on the host.
struct WtxRec {
    uint32_t tx_off;   // byte offset of the raw tx in the txraw blob (4-aligned)
    uint32_t tx_len;
    uint32_t in_base;  // first entry of this tx's inputs in the device input table
    uint32_t n_in;     // vin.size() as the host parsed it (table capacity)
};
struct WinJob {
    uint32_t tx;        // WtxRec index
    uint32_t nin;
    uint32_t code_off;  // compactsize || scriptCode in the code blob (4-aligned)
    uint32_t code_len;
    uint32_t hashtype;  // not SIGHASH_SINGLE (those keep the host preimage path)
    uint32_t row;       // tuple row whose msg receives the sighash
    uint32_t amount_lo, amount_hi;
};
static_assert(sizeof(WinJob) == 32, "WinJob: two 16-byte loads");

struct SighashJobs {
    pinned_bytes aux, pre;                          // padded messages, back to back
    std::vector<uint32_t> aux_off, aux_nblk;        // offsets / lengths in 64-byte blocks
    std::vector<uint32_t> pre_off, pre_nblk, pre_row;
    std::vector<PatchRec> patches;
    pinned_bytes tpl, code;                         // templates / code segments (4-aligned,
                                                    // templates followed by 8 zero bytes)
    std::vector<TplJob> tjobs;
    pinned_bytes txraw;                             // raw txs of the WinJobs (4-aligned)
    std::vector<WtxRec> wtx;
    std::vector<WinJob> wjobs;
    uint32_t win_entries = 0;                       // sum of WtxRec::n_in
    uint32_t add_wtx(const uint8_t* tx, size_t n, size_t n_in) {
        WtxRec r;
        r.tx_off = (uint32_t)txraw.size();
        r.tx_len = (uint32_t)n;
        r.in_base = win_entries;
        r.n_in = (uint32_t)n_in;
        txraw.insert(txraw.end(), tx, tx + n);
        txraw.resize(r.tx_off + ((n + 3) & ~(size_t)3), 0);
        win_entries += (uint32_t)n_in;
        wtx.push_back(r);
        return (uint32_t)wtx.size() - 1;
    }
    // the same from three pieces: a segwit tx without its marker, flag and witnesses (version ||
    // vin || vout || locktime: everything the BIP143 kernels read, at about half the bytes)
    uint32_t add_wtx3(const uint8_t* a, size_t na, const uint8_t* b, size_t nb, const uint8_t* c,
                      size_t nc, size_t n_in) {
        WtxRec r;
        const size_t n = na + nb + nc;
        r.tx_off = (uint32_t)txraw.size();
        r.tx_len = (uint32_t)n;
        r.in_base = win_entries;
        r.n_in = (uint32_t)n_in;
        txraw.insert(txraw.end(), a, a + na);
        txraw.insert(txraw.end(), b, b + nb);
        txraw.insert(txraw.end(), c, c + nc);
        txraw.resize(r.tx_off + ((n + 3) & ~(size_t)3), 0);
        win_entries += (uint32_t)n_in;
        wtx.push_back(r);
        return (uint32_t)wtx.size() - 1;
    }
    uint32_t add_tpl(const uint8_t* m, size_t n, const uint32_t* mid = nullptr) {
        return append_tpl(tpl, m, n, mid);
    }
    // compactsize(n) || m, 4-aligned: a scriptCode field (BIP143 / legacy serialization)
    uint32_t add_code_field(const uint8_t* m, size_t n) {
        const uint32_t off = (uint32_t)code.size();
        const size_t h = n < 253 ? 1 : n <= 0xFFFF ? 3 : 5;
        code.resize(off + ((h + n + 3) & ~(size_t)3), 0);
        uint8_t* o = &code[off];
        if (h == 1) {
            o[0] = (uint8_t)n;
        } else {
            o[0] = h == 3 ? 253 : 254;
            for (size_t i = 0; i + 1 < h; i++) o[1 + i] = (uint8_t)(n >> (8 * i));
        }
        if (n) memcpy(o + h, m, n);
        return off;
    }
    uint32_t add_code(const uint8_t* m, size_t n) {  // + a zero dword (K3' funnel reads)
        uint32_t off = (uint32_t)code.size();
        code.insert(code.end(), m, m + n);
        code.resize(off + ((n + 3) & ~(size_t)3) + 4, 0);
        return off;
    }
    static uint32_t tpl_nblk(uint32_t tpl_len, uint32_t code_len) {
        return (uint32_t)(sha_padded_len(tpl_len - 1 + code_len + 4) / 64);
    }
    uint32_t add_aux(const uint8_t* m, size_t n) {
        aux_off.push_back((uint32_t)(aux.size() / 64));
        sha_append_padded(aux, m, n);
        aux_nblk.push_back((uint32_t)(sha_padded_len(n) / 64));
        return (uint32_t)aux_off.size() - 1;
    }
    uint32_t add_pre(const uint8_t* m, size_t n, uint32_t row) {
        pre_off.push_back((uint32_t)(pre.size() / 64));
        sha_append_padded(pre, m, n);
        pre_nblk.push_back((uint32_t)(sha_padded_len(n) / 64));
        pre_row.push_back(row);
        return (uint32_t)pre_off.size() - 1;
    }
    void clear() {
        aux.clear(); pre.clear(); aux_off.clear(); aux_nblk.clear();
        pre_off.clear(); pre_nblk.clear(); pre_row.clear(); patches.clear();
        tpl.clear(); code.clear(); tjobs.clear();
        txraw.clear(); wtx.clear(); wjobs.clear(); win_entries = 0;
    }
};

// ECDSA tuple rows (big-endian 32-byte values).  msg rows whose sighash comes from a preimage
// are overwritten on the device by K3; constant ones (SIGHASH_SINGLE bug) are set by the host.
struct TupleRows {
    pinned_bytes tag, x, r, s;  // uploaded as they are (page-locked)
    std::vector<uint8_t> y, msg;
    // Producers that know may set these so that staging skips uploading rows (default: upload):
    // msg_one = every msg row is uint256 ONE (the rows the GPU sighash kernels do not overwrite
    // keep it; the device initialises the msg rows itself), y_unused = no 65-byte key (the y
    // rows are never read).  clear() resets both.
    bool msg_one = false, y_unused = false;
    // Key-hash conditions (the <20> OP_EQUALVERIFY of a P2WPKH / P2PKH spend taken over by the
    // device, engine.cpp DeferringChecker::defer_key_hash): row hrow[k] is valid only if
    // HASH160(its key) == hprog[20k, 20k + 20); the device ANDs that into the row's verdict.
    std::vector<uint32_t> hrow;
    pinned_bytes hprog;
    // Early Q halves (round 5, DeviceBatch::early_launch): emap[row] = the lane of the call's early
    // set whose (key, signature) bytes equal this row's, whose key half and Q ladder already ran
    // (K_keyq copies it instead of recomputing); rows past emap.size() or holding NO_EARLY have none.
    static constexpr uint32_t NO_EARLY = 0xFFFFFFFFu;
    std::vector<uint32_t> emap;
    void set_emap(size_t row, uint32_t e) {
        if (emap.size() <= row) emap.resize(row + 1, NO_EARLY);
        emap[row] = e;
    }
    void copy_emap(uint32_t* out, size_t lo, size_t hi) const { copy_map(emap, out, lo, hi); }
    // Early sighashes (TPL_EARLY): mmap[row] = the early row whose message (the same legacy
    // sighash job) the device copies into this row; NO_EARLY: none.
    std::vector<uint32_t> mmap;
    void set_mmap(size_t row, uint32_t e) {
        if (mmap.size() <= row) mmap.resize(row + 1, NO_EARLY);
        mmap[row] = e;
    }
    void copy_mmap(uint32_t* out, size_t lo, size_t hi) const { copy_map(mmap, out, lo, hi); }
    static void copy_map(const std::vector<uint32_t>& m, uint32_t* out, size_t lo, size_t hi) {
        const size_t have = std::min(std::max(m.size(), lo), hi);
        if (have > lo) memcpy(out, &m[lo], 4 * (have - lo));
        for (size_t k = have; k < hi; k++) out[k - lo] = NO_EARLY;
    }
    size_t size() const { return tag.size(); }
    // A row that stores its y / msg only when given: y32 == nullptr reads as zero (a 33-byte key),
    // m32 == nullptr as uint256 ONE.  y and msg may then hold only a prefix of the rows; readers
    // go through copy_y / copy_msg (or materialize() first).
    uint32_t add_lazy(uint8_t t, const uint8_t* x32, const uint8_t* r32, const uint8_t* s32,
                      const uint8_t* y32, const uint8_t* m32) {
        const size_t row = tag.size();
        tag.push_back(t);
        x.insert(x.end(), x32, x32 + 32);
        r.insert(r.end(), r32, r32 + 32);
        s.insert(s.end(), s32, s32 + 32);
        if (y32) {
            y.resize(32 * row, 0);
            y.insert(y.end(), y32, y32 + 32);
        }
        if (m32) {
            pad_msg(row);
            msg.insert(msg.end(), m32, m32 + 32);
        }
        return (uint32_t)row;
    }
    void pad_msg(size_t rows) {  // msg rows [msg.size() / 32, rows) = ONE
        size_t k = msg.size() / 32;
        if (k >= rows) return;
        msg.resize(32 * rows, 0);
        for (; k < rows; k++) msg[32 * k] = 1;
    }
    void materialize() {
        y.resize(32 * size(), 0);
        pad_msg(size());
    }
    void copy_y(uint8_t* out) const { copy_y(out, 0, size()); }  // 32 * size() bytes
    void copy_msg(uint8_t* out) const { copy_msg(out, 0, size()); }
    // rows [lo, hi) only, into out (= row lo's slot)
    void copy_y(uint8_t* out, size_t lo, size_t hi) const {
        const size_t have = std::min(std::max(y.size() / 32, lo), hi);  // stored rows in range end
        if (have > lo) memcpy(out, &y[32 * lo], 32 * (have - lo));
        if (hi > have) memset(out + 32 * (have - lo), 0, 32 * (hi - have));
    }
    void copy_msg(uint8_t* out, size_t lo, size_t hi) const {
        const size_t have = std::min(std::max(msg.size() / 32, lo), hi);
        if (have > lo) memcpy(out, &msg[32 * lo], 32 * (have - lo));
        for (size_t k = have; k < hi; k++) {
            memset(out + 32 * (k - lo), 0, 32);
            out[32 * (k - lo)] = 1;
        }
    }
    void add_key_hash(uint32_t row, const uint8_t* prog20) {
        hrow.push_back(row);
        hprog.insert(hprog.end(), prog20, prog20 + 20);
    }
    uint32_t add(uint8_t t, const uint8_t* x32, const uint8_t* y32, const uint8_t* r32,
                 const uint8_t* s32, const uint8_t* m32) {
        tag.push_back(t);
        x.insert(x.end(), x32, x32 + 32);
        y.insert(y.end(), y32, y32 + 32);
        r.insert(r.end(), r32, r32 + 32);
        s.insert(s.end(), s32, s32 + 32);
        msg.insert(msg.end(), m32, m32 + 32);
        return (uint32_t)tag.size() - 1;
    }
    void clear() {
        tag.clear(); x.clear(); y.clear(); r.clear(); s.clear(); msg.clear();
        hrow.clear(); hprog.clear(); emap.clear(); mmap.clear();
        msg_one = y_unused = false;
    }
};

// The device-built SigMsg path (sighash.hip taproot_tx_kernel / taproot_msg_kernel): per tx its
// bytes without marker / flag / witnesses and the serialized outputs it spends (both 4-aligned in
// txraw), per check a TapJob.
struct TtxRec {
    uint32_t tx_off, tx_len;  // the tx in txraw
    uint32_t sp_off, sp_len;  // the spent outputs (std::vector<CTxOut> serialization) in txraw
    uint32_t in_base, n_in;   // input table entries [in_base, in_base + n_in)
    uint32_t pad[2];
};
struct TapJob {
    uint32_t ttx, nin, hash_type;
    uint32_t spend_type;  // (ext_flag << 1) | annex present (interpreter.cpp:1534)
    uint32_t row;         // BIP340 row whose msg receives the sighash
    uint32_t ext_off;     // byte offset in the ext blob: [sha_annex] [sha_single_output] [tapleaf]
    uint32_t codesep;     // BIP342 codesep_pos
    uint32_t flags;       // 1: BIP342 (tapleaf hash, key_version, codesep_pos follow)
};
struct TaprootTxJobs {
    std::vector<uint8_t> txraw, ext;
    std::vector<TtxRec> ttx;
    std::vector<TapJob> jobs;
    uint32_t in_entries = 0;
    void clear() {
        txraw.clear(); ext.clear(); ttx.clear(); jobs.clear(); in_entries = 0;
    }
    void put_raw(const uint8_t* p, size_t n) {
        txraw.insert(txraw.end(), p, p + n);
    }
    void align4() { txraw.resize((txraw.size() + 3) & ~(size_t)3, 0); }
};

// BIP341 / BIP342 signature checks (host/taproot.cpp): single-SHA256 aux messages (a tx's
// sha_prevouts / sha_amounts / sha_scriptpubkeys / sha_sequences / sha_outputs, a check's
// sha_annex / sha_single_output), SigMsg messages hashed as TapSighash tagged hashes (the
// 64-byte tag block is the kernel's starting midstate) with the aux digests patched in, and the
// BIP340 rows (sig64, x-only key) their digests feed.
struct TaprootJobs {
    std::vector<uint8_t> aux, msg;                   // padded messages, back to back
    std::vector<uint32_t> aux_off, aux_nblk;         // in 64-byte blocks
    std::vector<uint32_t> msg_off, msg_nblk, msg_row;
    std::vector<PatchRec> patches;                   // aux digest -> msg blob byte offset
    std::vector<uint8_t> sig64, pk32;                // BIP340 rows
    TaprootTxJobs dev;                               // device-built SigMsgs (the default path)
    size_t rows() const { return pk32.size() / 32; }
    void clear() {  // keeps the capacity (a caller's next round reuses it)
        aux.clear(); msg.clear(); aux_off.clear(); aux_nblk.clear(); msg_off.clear();
        msg_nblk.clear(); msg_row.clear(); patches.clear(); sig64.clear(); pk32.clear();
        dev.clear();
    }
    uint32_t add_aux(const uint8_t* m, size_t n) {
        aux_off.push_back((uint32_t)(aux.size() / 64));
        sha_append_padded(aux, m, n);
        aux_nblk.push_back((uint32_t)(sha_padded_len(n) / 64));
        return (uint32_t)aux_off.size() - 1;
    }
    uint32_t add_msg(const uint8_t* m, size_t n, uint32_t row) {
        msg_off.push_back((uint32_t)(msg.size() / 64));
        sha_append_padded(msg, m, n, 64);
        msg_nblk.push_back((uint32_t)(sha_padded_len(n) / 64));
        msg_row.push_back(row);
        return (uint32_t)msg_off.size() - 1;
    }
};

// SHA256(tag) || SHA256(tag) compressed from the IV: the starting midstate of the TapSighash
// tagged hash (host/taproot.cpp computes it once).
void tapsighash_midstate(uint32_t out[8]);

// Stage + run + fetch on `device` (synchronous): BIP341 sighashes (msg32_out, optional, 32 bytes
// per row) and BIP340 verdicts (1 valid).
int gpu_taproot_verify(int device, const TaprootJobs& jobs, uint8_t* verdict, uint8_t* msg32_out);
// The same over the concatenation of P parts (rows in part order).
int gpu_taproot_verify_parts(int device, const TaprootJobs* const* parts, size_t P,
                             uint8_t* verdict, uint8_t* msg32_out);
// The same in two phases on one of TAPROOT_SLOTS contexts per (thread, device): begin stages,
// uploads and launches on `slot`'s stream and returns; end waits for it and copies the verdicts
// (and, with msg32_out, the sighashes) back.  The pipelined bcc_taproot_verify_batch rotates the
// slots (two rounds in flight while the host builds a third), so a round's upload runs beside the
// previous round's kernels.  Each begin is matched by an end.
constexpr int TAPROOT_SLOTS = 3;
int gpu_taproot_begin(int device, int slot, const TaprootJobs* const* parts, size_t P);
int gpu_taproot_end(int device, int slot, uint8_t* verdict, uint8_t* msg32_out);

// Device scratch of the signature kernels: s^-1 rows (ECDSA) and, for one chunk of lanes, the
// Q tables + ladder states.  Every synchronous entry point owns one per (thread, device), so
// concurrent callers never share scratch (the reference ABI is reentrant).  Launches
// that share a scratch must be ordered (one stream).
struct SigScratch {
    int dev = -1;
    void* sinv = nullptr;
    size_t sinv_cap = 0;   // tuples
    void* chunk = nullptr;
    size_t chunk_cap = 0;  // lanes
    size_t chunk_short = 0;  // a chunk request the device could not hold (served by chunk_cap)
    size_t key_ready = 0;  // tuples whose key half of the prep ran ahead (ecdsa_launch_key)
    size_t q_ready = 0;    // tuples whose Q ladder ran ahead (ecdsa_launch_q)
    void* qtab2 = nullptr;  // the Q tables of K_keyq's latency mode (two lanes per tuple)
    size_t qtab2_cap = 0;   // lanes
    // Round 6, the residency tail: K_keyq of a launch that is not a whole number of residency
    // rounds runs as two launches, [0, q_split) and [q_split, q_ready); ev_qa is recorded after
    // the first, so the G ladder of those lanes can fill the idle slots of the second's last
    // round (ecdsa_launch_after_pre).  aux / ev_ga: the second stream of the single-stream form.
    size_t q_split = 0;
    void* ev_qa = nullptr;
    void* ev_ga = nullptr;
    void* aux = nullptr;
    SigScratch() = default;
    SigScratch(const SigScratch&) = delete;
    SigScratch& operator=(const SigScratch&) = delete;
    ~SigScratch();
};

// Asynchronous launches of the ECDSA / BIP340 kernels on `stream` with caller-owned scratch
// (grown here when needed; growing synchronises the device).  Return 0 or a hipError_t value.
int ecdsa_launch(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                 const uint8_t* d_r, const uint8_t* d_s, const uint8_t* d_m, uint8_t* d_verdict,
                 size_t n, void* stream);
// The same in two parts: K_inv + K_key (s^-1 and the pubkey parse / decompression read only the
// s and key rows, so they can run beside the sighash kernels on another stream) and everything
// after them (must be ordered after both, and after the sighash kernels that write m).
int ecdsa_launch_pre(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x,
                     const uint8_t* d_y, const uint8_t* d_s, size_t n, void* stream);
// The message-free part of the ECDSA lane ahead of the sighash kernels, in one launch
// (twist_keyq_kernel): the key half of the prep (key parse without a square root, the co-Z Q_w
// table), the r / s half (u2 = r s^-1, GLV split) and the Q ladder B = u2 Q_w, on `stream` after
// K_inv (ecdsa_launch_pre for the same n, ordered before it).  ecdsa_launch_key marks the round
// (no launch; it may be called from any stream); the next ecdsa_launch_after_pre for the same n
// then forms u1 from the sighash rows and runs only the G ladder, the combine and K_tfin.  Both
// are no-ops (return 0) when n does not fit one scratch chunk (the chunked path preps per chunk).
int ecdsa_launch_key(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                     size_t n, void* stream);
int ecdsa_launch_q(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                   const uint8_t* d_r, const uint8_t* d_s, size_t n, void* stream);
// The same for rows that may have an early twin (TupleRows::emap, device copy d_emap): a mapped
// row's key half and Q ladder are copied from lane emap[row] of `early` (an ecdsa_launch_q over
// the call's early set, ordered before this on `stream`); K_keyq computes only the others.
int ecdsa_launch_q_mapped(SigScratch& sc, const SigScratch& early, size_t early_n,
                          const uint32_t* d_emap, const uint8_t* d_tag, const uint8_t* d_x,
                          const uint8_t* d_y, const uint8_t* d_r, const uint8_t* d_s, size_t n,
                          void* stream);
// ev_rows_read (optional hipEvent_t) is recorded on `stream` once the last kernel that reads the
// s / m / key rows and the s^-1 rows has been launched (the prep kernel): later writers of those
// rows (the next run's front kernels) need only wait for it, not for the ladder.
// verdict_and: the caller has set d_verdict[0, n) to 1 (and may already have cleared rows, e.g.
// the key-hash conditions); K_tfin then only clears the rows that fail.
// ev_q_done (optional hipEvent_t): recorded after the Q launches on another stream; `stream`
// waits for it before the lanes that need it (with a split K_keyq, only the G ladder of the tail
// lanes waits: the full rounds' G ladder goes first, beside the tail's K_keyq).
int ecdsa_launch_after_pre(SigScratch& sc, const uint8_t* d_tag, const uint8_t* d_x,
                           const uint8_t* d_y, const uint8_t* d_r, const uint8_t* d_s,
                           const uint8_t* d_m, uint8_t* d_verdict, size_t n, void* stream,
                           void* ev_rows_read = nullptr, bool verdict_and = false,
                           void* ev_q_done = nullptr);
int schnorr_launch(SigScratch& sc, const uint8_t* d_sig64, const uint8_t* d_msg32,
                   const uint8_t* d_xonly32, uint8_t* d_verdict, size_t n, void* stream);

// Raw CPubKey::Verify tuples of bcc_pubkey_verify_batch (round 5): the caller's blobs as they are,
// parsed on the device by K_der (der.hip: the length filter, lax DER, r / s == 0) into the rows the
// ECDSA kernels read, so that the host only copies bytes.  Offsets are absolute (n + 1 each).
struct DerTuples {
    const uint8_t* pub_blob = nullptr;
    const uint64_t* pub_off = nullptr;
    const uint8_t* msg32 = nullptr;
    const uint8_t* sig_blob = nullptr;
    const uint64_t* sig_off = nullptr;
    size_t n = 0;
    uint64_t pub_bytes() const { return pub_off[n] - pub_off[0]; }
    uint64_t sig_bytes() const { return sig_off[n] - sig_off[0]; }
};
// K_der over n tuples whose blobs / offsets are in HBM (blob bytes [0, *_bytes) hold offsets
// [*_base, *_base + *_bytes)): rows tag / x / y / r / s.
int der_launch(const uint8_t* pub, const uint64_t* pub_off, uint64_t pub_base, uint64_t pub_bytes,
               const uint8_t* sig, const uint64_t* sig_off, uint64_t sig_base, uint64_t sig_bytes,
               size_t n, uint8_t* tag, uint8_t* x, uint8_t* y, uint8_t* r, uint8_t* s, void* stream);

// Device-resident batch (one per device / per caller thread).  stage() uploads, run() only
// launches kernels (graph-capturable: no allocation, no synchronisation, once the scratch has
// grown to the batch).  A null stream means the batch's own non-blocking stream.
// Messages that are known only after a round's launches: the long SHA chains hashed on the host
// while the device runs the message-independent kernels (engine.cpp, bcc_set_host_chain_blocks).
// Called once those kernels are queued; appends batch-local rows and their 32-byte digests.  The
// G ladder (the first kernel that reads a message) waits for them.
using LateMsgFill = std::function<void(std::vector<uint32_t>& rows, std::vector<uint8_t>& digs)>;

class DeviceBatch {
public:
    explicit DeviceBatch(int device);
    ~DeviceBatch();
    int stage(const SighashJobs& jobs, const TupleRows& rows);
    // the concatenation of P parts (row / message / job indices fixed up per part)
    // direct: the parts' page-locked arrays go up as they are (set_direct_upload), so they must
    // stay unchanged until the round has run; false copies everything into the pinned image
    int stage_parts(const SighashJobs* const* jobs, const TupleRows* const* rows, size_t P,
                    bool direct = false);
    // Rows uploaded per host shard while the host pass still runs (round 6): pre_arm on the
    // calling thread before the pass (P shards of at most cap_rows rows), pre_upload by the worker
    // that finished shard t (its tag / x / r / s to the shard's own HBM buffer, on the batch's
    // pre stream); stage_parts then gathers them into the arena with K_rowgather instead of
    // uploading them (falling back to the upload for a shard that did not fit or was not sent).
    // The rows must stay unchanged until the round has run, as with the direct upload.
    int pre_arm(unsigned P, size_t cap_rows);
    void pre_upload(unsigned t, const TupleRows& rows);
    // raw tuples (DerTuples): blobs, offsets and messages staged; run() starts with K_der
    int stage_der(const DerTuples& t);
    int run(void* stream, const LateMsgFill* late = nullptr);  // K1..K4
    int run_sighash(void* stream);               // K1..K3 only
    int run_ecdsa(void* stream);                 // K4 only
    int fetch_verdicts(uint8_t* out);            // synchronous D2H (waits for the last run)
    int fetch_msgs(uint8_t* out);                // synchronous D2H (tests)
    size_t n_tuples() const { return n_rows_; }
    size_t n_key_hashes() const { return n_hash_; }  // TupleRows::hrow conditions staged
    size_t n_pre() const { return n_pre_ + n_tjob_ + n_wjob_; }  // sighash messages (all kinds)
    size_t n_wtx() const { return n_wtx_; }
    // Algorithmic bytes of one run of the sighash stage: padded messages + digests of the host-built
    // jobs, and raw tx bytes + job records + scriptCode fields + per-tx hashes + sighashes of the
    // device-built BIP143 jobs.
    size_t sighash_bytes() const { return sighash_bytes_; }
    size_t n_aux() const { return n_aux_; }
    size_t pre_blocks() const { return pre_blocks_ + tjob_blocks_; }
    size_t aux_blocks() const { return aux_blocks_; }
    int device() const { return dev_; }
    // raw device pointers (bench / profiling)
    uint8_t *d_tag = nullptr, *d_x = nullptr, *d_y = nullptr, *d_r = nullptr, *d_s = nullptr,
            *d_m = nullptr, *d_v = nullptr;

private:
    int sync();
    void* pick(void* stream);
    int launch_front(struct ihipStream_t* st);        // K_wtx + K3' + K1 fused, then the rest
    // part 1: the tuple rows (and the pre-uploaded rows' gather), part 2: the rest; 3: both
    int upload_on(struct ihipStream_t* rows_stream, struct ihipStream_t* rest_stream, int part = 3);
    bool up_pending_ = false;      // the staged image is not on the device yet (issued by run)
    struct UpCopy {  // one host -> HBM copy of the pending upload
        size_t dst;      // arena offset
        const void* src; // the pinned image or a part's own page-locked array
        size_t len;
        bool rows;       // a tuple-row region (the ECDSA stream's) or a sighash input
    };
    std::vector<UpCopy> up_copies_;
    bool up_msg_one_ = false;      // the msg rows are set to ONE with the upload
    // per-shard row pre-upload (pre_arm / pre_upload): shard t's tag | x | r | s at pre_buf_[t]
    static constexpr unsigned PRE_MAX_SHARDS = 64;
    std::vector<uint8_t*> pre_buf_;
    size_t pre_cap_ = 0;               // rows per shard buffer
    std::vector<size_t> pre_rows_;     // rows sent per shard (SIZE_MAX: none)
    unsigned pre_P_ = 0;
    bool pre_armed_ = false;
    void* pre_stream_ = nullptr;       // hipStream_t of the pre-uploads
    void* ev_pre_ = nullptr;           // hipEvent_t: every pre-upload issued so far is done
    bool gather_pending_ = false;      // the next run gathers the pre-uploaded rows (upload_on)
    std::vector<size_t> gather_row0_;  // the shards' first rows in the arena (P + 1)
    int launch_after_front(struct ihipStream_t* st);  // K_win, K2, K3
    int launch_key_hash(struct ihipStream_t* st);     // K_h160: key-hash conditions into the verdicts
    int run_stages(void* stream, const LateMsgFill* late);
    int put_late(struct ihipStream_t* st, const LateMsgFill* late);  // late rows -> d_m (K_late)
    std::vector<uint32_t> late_rows_;
    std::vector<uint8_t> late_digs_;
    void* late_host_ = nullptr;  // pinned: rows then digests
    uint8_t* late_dev_ = nullptr;
    size_t late_cap_ = 0;        // entries of late_host_ / late_dev_
    bool kh_done_ = false;  // run_stages ran K_h160 already (ahead of the ladder, verdict_and)
    int dev_;
    void* own_stream_ = nullptr;   // hipStream_t, created on first use
    void* last_stream_ = nullptr;  // stream of the last run
    void* side_stream_ = nullptr;  // the key / Q-ladder chain beside the sighash kernels (run())
    void* ev_fork_ = nullptr;      // hipEvent_t: run() start on the main stream
    void* ev_join_ = nullptr;      // hipEvent_t: the Q ladder done on the side stream
    void* ev_up_ = nullptr;        // hipEvent_t: the tuple rows uploaded (side stream)
    void* ev_rows_up_ = nullptr;   // hipEvent_t: upload_on's row copies done (the rest waits)
    void* ev_block_ = nullptr;     // hipEvent_t (blocking sync): host waits sleep, not spin
    int wait(void* stream);
    SigScratch scratch_;
    void* arena_ = nullptr;
    size_t cap_ = 0;
    void* host_image_ = nullptr;  // pinned host image of the arena (staging)
    size_t host_cap_ = 0;
    void* vbuf_ = nullptr;        // pinned verdict buffer (fetch_verdicts)
    size_t vcap_ = 0;
    // Round 5: the verdicts reach vbuf_ through a kernel queued behind the round's last kernel
    // (queue_verdicts), not a copy-engine D2H issued at fetch time, which waited in the one copy
    // queue behind the next pipelined round's upload
    void* vbuf_dev_ = nullptr;    // vbuf_ as the device addresses it
    bool v_queued_ = false;       // the current run's verdicts are on their way to vbuf_
    int ensure_vbuf();            // vbuf_ for n_rows_ (stage time: run() allocates nothing)
    int queue_verdicts(struct ihipStream_t* st);
    size_t n_rows_ = 0, n_pre_ = 0, n_aux_ = 0, n_patch_ = 0, pre_blocks_ = 0, aux_blocks_ = 0;
    uint8_t *d_aux_ = nullptr, *d_pre_ = nullptr, *d_auxd_ = nullptr;
    uint32_t *d_aux_off_ = nullptr, *d_aux_nblk_ = nullptr, *d_pre_off_ = nullptr,
             *d_pre_nblk_ = nullptr, *d_pre_row_ = nullptr;
    PatchRec* d_patch_ = nullptr;
    size_t n_tjob_ = 0, tjob_blocks_ = 0;
    uint8_t *d_tpl_ = nullptr, *d_code_ = nullptr;
    TplJob* d_tjob_ = nullptr;
    size_t n_wtx_ = 0, n_wjob_ = 0, n_win_ = 0, sighash_bytes_ = 0;
    uint8_t *d_txraw_ = nullptr, *d_txd_ = nullptr, *d_zeros_ = nullptr;
    WtxRec* d_wtx_ = nullptr;
    WinJob* d_wjob_ = nullptr;
    uint32_t* d_intab_ = nullptr;
    size_t n_hash_ = 0;
    uint32_t* d_hrow_ = nullptr;
    uint8_t* d_hprog_ = nullptr;
    uint32_t* d_emap_ = nullptr;  // staged TupleRows::emap (null: no row has an early twin)
    uint32_t* d_mmap_ = nullptr;  // staged TupleRows::mmap (null: no row takes an early sighash)
    // stage_der: the rows come from K_der over these (n_der_ = 0: rows staged by stage_parts)
    size_t n_der_ = 0;
    const uint8_t *d_pub_ = nullptr, *d_sig_ = nullptr;
    const uint64_t *d_pub_off_ = nullptr, *d_sig_off_ = nullptr;
    uint64_t pub_base_ = 0, pub_bytes_ = 0, sig_base_ = 0, sig_bytes_ = 0;

public:
    // Early Q halves (round 5): the key half, u2 and the Q ladder (K_inv + K_keyq) of a call's
    // pre-extracted (key, signature) rows, launched on a stream of their own while the host still
    // interprets the call; a later round whose rows carry TupleRows::emap copies them instead of
    // running its own K_keyq on those rows.  early_reset forgets the set (a new call).
    // jobs (optional, one per part): legacy template jobs whose rows are the early rows of the same
    // part (early sighashes, TPL_EARLY), hashed on a stream of their own
    int early_launch(const TupleRows* const* rows, size_t P, const SighashJobs* const* jobs = nullptr);
    void early_reset();
    size_t early_rows() const { return early_n_; }

private:
    void* early_stream_ = nullptr;  // hipStream_t
    void* ev_early_ = nullptr;      // hipEvent_t: the early K_keyq done
    bool early_pending_ = false;    // ev_early_ recorded and maybe not reached yet
    size_t early_n_ = 0;            // rows of the current early set (0: none)
    SigScratch early_scratch_;
    void* early_arena_ = nullptr;   // tag | x | y | r | s rows of the early set
    size_t early_cap_ = 0;
    void* early_host_ = nullptr;    // pinned image of early_arena_
    size_t early_host_cap_ = 0;
    void* early_sig_stream_ = nullptr;  // hipStream_t: the early sighash jobs
    void* ev_early_up_ = nullptr;       // hipEvent_t: the early image uploaded
    void* ev_early_sig_ = nullptr;      // hipEvent_t: the early sighashes done
    bool early_msgs_ = false;           // the current early set has sighashes (early_msg_)
    uint8_t* early_msg_ = nullptr;      // 32 bytes per early row (only job rows written)
};

// The calling thread's device batch on `device` (the one gpu_verify_parts runs): early Q halves
// for the call's pre-extracted rows (DeviceBatch::early_launch), and the reset of a new call.
int gpu_early_launch(int device, const TupleRows* const* rows, size_t P,
                     const SighashJobs* const* jobs = nullptr);
void gpu_early_reset(int device);

// Threads the calling thread's device batches use to fill their pinned staging image (0: one per
// part, the default).  The batch engine lowers it on its pipeline worker, whose staging runs
// beside the host pass: the GPU box's CPU share is a CFS quota, and threads beyond it are
// throttled for the rest of the quota period.
void set_stage_threads(unsigned n);

// Direct upload (round 6, default on; bcc_set_direct_upload, BCC_DIRECT_UPLOAD=0 turns it off):
// DeviceBatch::stage_parts sends the parts' page-locked arrays (tuple rows, raw txs, sighash
// blobs, key-hash programs) to HBM as they are, one copy per part and array, and fills the pinned
// image only with the records it rebases.  Off: every array is copied into the image first.
void set_direct_upload(bool on);
bool direct_upload();

// Free the calling thread's cached device state: the verify_batch / Taproot device batches and
// contexts (sighash.hip) and the tuple-path contexts (ecdsa_verify.hip).
void release_device_thread_state();
void release_tuple_thread_state();

// One-shot helper: stage + run + fetch on `device` (synchronous).
// *stage_seconds (optional) receives the host -> HBM staging time.
int gpu_verify_batch(int device, const SighashJobs& jobs, const TupleRows& rows, uint8_t* verdict,
                     double* stage_seconds = nullptr);
// The same over the concatenation of `parts` (jobs[p], rows[p]) pairs: verdict rows in order.
// A device round staged by one thread and run by another (the pipelined verify_batch: the caller
// fills the pinned image with its whole team, the pipeline worker uploads, launches and waits).
// The object keeps its device batch (arena, pinned image, scratch, streams) for reuse.
struct StagedRound;
StagedRound* gpu_staged_new(int device);
void gpu_staged_free(StagedRound* s);
// Fills s's pinned image from the parts, which must stay unchanged until gpu_staged_run /
// gpu_staged_finish returns: with direct upload the launch's copies read their arrays.
int gpu_staged_stage(StagedRound* s, const SighashJobs* const* jobs, const TupleRows* const* rows,
                     size_t parts, double* stage_seconds);
// Per-shard row pre-upload on s's batch (DeviceBatch::pre_arm / pre_upload): armed by the caller
// before a host pass of P shards, sent by each shard's worker when its rows are final.
int gpu_staged_pre_arm(StagedRound* s, unsigned P, size_t cap_rows);
void gpu_staged_pre_upload(StagedRound* s, unsigned t, const TupleRows& rows);
// Fills s's pinned image with raw tuples (DeviceBatch::stage_der; the caller's buffers are copied).
int gpu_staged_stage_der(StagedRound* s, const DerTuples& t, double* stage_seconds);
// One synchronous round of raw tuples on the calling thread's batch of `device`.
int gpu_verify_der(int device, const DerTuples& t, uint8_t* verdict);
// Runs the staged round on the calling thread (any thread): verdict rows in order.  On an error
// the batch is dropped (the next stage starts from a fresh one).
int gpu_staged_run(StagedRound* s, uint8_t* verdict, const LateMsgFill* late);
// The same in two phases: launch uploads and queues the kernels and returns; finish waits and
// copies the verdicts.  Two staged rounds in flight overlap one's upload with the other's kernels.
int gpu_staged_launch(StagedRound* s, const LateMsgFill* late);
int gpu_staged_finish(StagedRound* s, uint8_t* verdict);

// `late` (optional): rows whose message the host delivers after the launches (LateMsgFill).
int gpu_verify_parts(int device, const SighashJobs* const* jobs, const TupleRows* const* rows,
                     size_t parts, uint8_t* verdict, double* stage_seconds = nullptr,
                     const LateMsgFill* late = nullptr);

}  // namespace bcc
