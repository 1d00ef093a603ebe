// oracle/ref_shim.cpp — TEST INFRASTRUCTURE ONLY (never linked into the product).
//
// A thin C-ABI shim over the *reference* libbitcoinconsensus + libsecp256k1, compiled from the
// unmodified sources under /root/reference by oracle/Makefile into oracle/_ref/libref_consensus.so.
// It exposes the reference's own per-signature semantics so that tests/, smoke() and bench.py's
// cpu_baseline leg can use the reference as the checker / CPU baseline:
//
//   * ref_pubkey_verify   -> CPubKey(pub).Verify(hash, sig)          depend/bitcoin/src/pubkey.cpp:191-207
//                            (lax DER + normalize-S + secp256k1_ecdsa_verify)
//   * ref_capture_script  -> VerifyScript with a checker that records every
//                            (pubkey, sig, sighash, verdict) the interpreter asks for
//                            (GenericTransactionSignatureChecker::VerifyECDSASignature,
//                             depend/bitcoin/src/script/interpreter.cpp:1644-1676)
//   * ref_schnorr_verify  -> secp256k1_schnorrsig_verify            secp256k1/src/modules/schnorrsig/main_impl.h:190-237
//   * ref_taproot_check   -> GenericTransactionSignatureChecker::CheckSchnorrSignature with the
//                            tx's PrecomputedTransactionData initialised with its spent outputs
//                            (interpreter.cpp:1422-1472, 1491-1574, 1678-1704); the signature hash
//                            is captured at VerifySchnorrSignature
//   * ref_check_sighash   -> SignatureHash as CheckECDSASignature computes it for one check
//                            (interpreter.cpp:1576-1642, 1656-1676)
//   * ref_sign / ref_pubkey_create / ref_schnorr_sign: fixture generation only
//   * ref_bench_* / ref_bulk_* -> dynamically chunked std::thread pool over the reference entry
//                            points (cpu_baseline timing, bulk agreement checks)
//
// The shim contains no consensus logic of its own: every verdict comes from the reference.
#include <script/bitcoinconsensus.h>
#include <script/interpreter.h>
#include <primitives/transaction.h>
#include <hash.h>
#include <pubkey.h>
#include <version.h>
#include <secp256k1.h>
#include <secp256k1_schnorrsig.h>
#include <secp256k1_extrakeys.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

secp256k1_context* sign_ctx() {
    static secp256k1_context* ctx =
        secp256k1_context_create(SECP256K1_CONTEXT_SIGN | SECP256K1_CONTEXT_VERIFY);
    return ctx;
}

// Minimal byte-reader with the Unserialize stream interface (avoids CDataStream, whose
// allocator pulls support/cleanse.cpp, which build.rs does not compile).
class ByteReader {
public:
    ByteReader(const unsigned char* p, size_t n) : m_p(p), m_n(n) {}
    void read(char* dst, size_t k) {
        if (k > m_n) throw std::ios_base::failure("end of data");
        memcpy(dst, m_p, k);
        m_p += k;
        m_n -= k;
    }
    template <typename T> ByteReader& operator>>(T&& obj) {
        ::Unserialize(*this, obj);
        return *this;
    }
    int GetVersion() const { return PROTOCOL_VERSION; }
    int GetType() const { return SER_NETWORK; }

private:
    const unsigned char* m_p;
    size_t m_n;
};

struct Capture {
    std::vector<unsigned char> pub, sig;  // sig without the hashtype byte
    uint256 sighash;
    bool verdict;
};

class CapturingChecker : public TransactionSignatureChecker {
public:
    mutable std::vector<Capture> log;
    CapturingChecker(const CTransaction* tx, unsigned int nIn, const CAmount& amount,
                     const PrecomputedTransactionData& txdata)
        : TransactionSignatureChecker(tx, nIn, amount, txdata) {}

protected:
    bool VerifyECDSASignature(const std::vector<unsigned char>& vchSig, const CPubKey& pubkey,
                              const uint256& sighash) const override {
        bool ok = TransactionSignatureChecker::VerifyECDSASignature(vchSig, pubkey, sighash);
        log.push_back(Capture{std::vector<unsigned char>(pubkey.begin(), pubkey.end()), vchSig,
                              sighash, ok});
        return ok;
    }
};

class SchnorrCapturingChecker : public TransactionSignatureChecker {
public:
    mutable uint256 sighash;
    mutable bool called = false;
    SchnorrCapturingChecker(const CTransaction* tx, unsigned int nIn, const CAmount& amount,
                            const PrecomputedTransactionData& txdata)
        : TransactionSignatureChecker(tx, nIn, amount, txdata) {}

protected:
    bool VerifySchnorrSignature(Span<const unsigned char> sig, const XOnlyPubKey& pubkey,
                                const uint256& h) const override {
        sighash = h;
        called = true;
        return TransactionSignatureChecker::VerifySchnorrSignature(sig, pubkey, h);
    }
};

// ---- CPU baseline timing: std::thread pool with DYNAMIC chunking ----
// Workers pull chunks of CHUNK consecutive items from one atomic counter (rayon's work stealing
// restated for a flat index space), so one long item (a many-input legacy tx) does not leave the
// other threads idle behind a static partition.  Returns wall seconds; the per-item results are
// written so the caller can cross-check verdicts.
constexpr long CHUNK = 64;

template <class F>
double run_pool(int nthreads, long n, F f) {
    auto t0 = std::chrono::steady_clock::now();
    std::atomic<long> next{0};
    std::vector<std::thread> pool;
    auto worker = [&]() {
        for (;;) {
            long lo = next.fetch_add(CHUNK, std::memory_order_relaxed);
            if (lo >= n) break;
            long hi = lo + CHUNK < n ? lo + CHUNK : n;
            for (long i = lo; i < hi; ++i) f(i);
        }
    };
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
    worker();
    for (auto& th : pool) th.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace

extern "C" {

int ref_version() { return (int)bitcoinconsensus_version(); }

int ref_verify_script_with_amount(const unsigned char* spk, unsigned int spklen, int64_t amount,
                                  const unsigned char* tx, unsigned int txlen, unsigned int nIn,
                                  unsigned int flags, int* err) {
    bitcoinconsensus_error e = bitcoinconsensus_ERR_OK;
    int r = bitcoinconsensus_verify_script_with_amount(spk, spklen, amount, tx, txlen, nIn, flags, &e);
    if (err) *err = (int)e;
    return r;
}

int ref_verify_script(const unsigned char* spk, unsigned int spklen, const unsigned char* tx,
                      unsigned int txlen, unsigned int nIn, unsigned int flags, int* err) {
    bitcoinconsensus_error e = bitcoinconsensus_ERR_OK;
    int r = bitcoinconsensus_verify_script(spk, spklen, tx, txlen, nIn, flags, &e);
    if (err) *err = (int)e;
    return r;
}

// CPubKey::Verify semantics: pub = 33/65 serialized bytes, hash32 = raw sighash bytes
// (uint256::begin()), sig = DER signature WITHOUT the hashtype byte.
int ref_pubkey_verify(const unsigned char* pub, size_t publen, const unsigned char* hash32,
                      const unsigned char* sig, size_t siglen) {
    CPubKey key(pub, pub + publen);
    uint256 h(std::vector<unsigned char>(hash32, hash32 + 32));
    std::vector<unsigned char> vs(sig, sig + siglen);
    return key.Verify(h, vs) ? 1 : 0;
}

// Runs the reference VerifyScript on (spk, tx, nIn, amount, flags) with a capturing checker.
// Writes up to `cap` records into the out arrays: pub (65 B slot + len), sig (80 B slot + len),
// sighash (32 B raw), verdict. Returns the script result (1/0), or -1 on deserialize error.
int ref_capture_script(const unsigned char* spk, unsigned int spklen, int64_t amount,
                       const unsigned char* txb, unsigned int txlen, unsigned int nIn,
                       unsigned int flags, int cap, unsigned char* pub65, int* publen,
                       unsigned char* sig80, int* siglen, unsigned char* hash32, int* verdict,
                       int* ncaptured, int* script_error) {
    try {
        ByteReader ss(txb, txlen);
        CTransaction tx(deserialize, ss);
        if (nIn >= tx.vin.size()) return -2;
        PrecomputedTransactionData txdata(tx);
        CapturingChecker chk(&tx, nIn, amount, txdata);
        ScriptError serr = SCRIPT_ERR_OK;
        bool ok = VerifyScript(tx.vin[nIn].scriptSig, CScript(spk, spk + spklen),
                               &tx.vin[nIn].scriptWitness, flags, chk, &serr);
        int n = 0;
        for (const auto& c : chk.log) {
            if (n >= cap) break;
            memset(pub65 + 65 * n, 0, 65);
            memset(sig80 + 80 * n, 0, 80);
            memcpy(pub65 + 65 * n, c.pub.data(), c.pub.size() > 65 ? 65 : c.pub.size());
            publen[n] = (int)c.pub.size();
            size_t sl = c.sig.size() > 80 ? 80 : c.sig.size();
            memcpy(sig80 + 80 * n, c.sig.data(), sl);
            siglen[n] = (int)c.sig.size();
            memcpy(hash32 + 32 * n, c.sighash.begin(), 32);
            verdict[n] = c.verdict ? 1 : 0;
            ++n;
        }
        *ncaptured = (int)chk.log.size();
        if (script_error) *script_error = (int)serr;
        return ok ? 1 : 0;
    } catch (const std::exception&) {
        return -1;
    }
}

int ref_schnorr_verify(const unsigned char* sig64, const unsigned char* msg32,
                       const unsigned char* xonly32) {
    secp256k1_xonly_pubkey pk;
    if (!secp256k1_xonly_pubkey_parse(sign_ctx(), &pk, xonly32)) return 0;
    return secp256k1_schnorrsig_verify(sign_ctx(), sig64, msg32, &pk);
}

// CheckSchnorrSignature (interpreter.cpp:1678-1704) for input nIn of tx, whose spent outputs are
// the serialized std::vector<CTxOut> `spent` (PrecomputedTransactionData::Init).  sigversion 0 =
// TAPROOT, 1 = TAPSCRIPT.  annex (incl. its 0x50 byte) or NULL; its hash is formed as
// VerifyWitnessProgram does (:1889-1893).  Returns 1 / 0 (with *serror), or -1 if the tx / spent
// outputs do not deserialize, their counts differ or nIn is out of range (the reference asserts).
// *hashed = 1 when the signature hash was computed (then written to sighash32).
int ref_taproot_check(const unsigned char* txb, size_t txlen, const unsigned char* spent,
                      size_t spentlen, unsigned int nIn, const unsigned char* sig, size_t siglen,
                      const unsigned char* pk32, int sigversion, const unsigned char* annex,
                      size_t annexlen, const unsigned char* tapleaf32, uint32_t codesep_pos,
                      int* serror, unsigned char* sighash32, int* hashed) {
    try {
        ByteReader ss(txb, txlen);
        CTransaction tx(deserialize, ss);
        std::vector<CTxOut> outs;
        ByteReader so(spent, spentlen);
        so >> outs;
        unsigned char extra;
        bool trailing = true;
        try { so.read((char*)&extra, 1); } catch (const std::exception&) { trailing = false; }
        if (trailing || outs.size() != tx.vin.size() || nIn >= tx.vin.size()) return -1;
        // the tx must be exactly tx_len bytes (bitcoinconsensus.cpp:91-92's size rule)
        if (GetSerializeSize(tx, PROTOCOL_VERSION) != txlen) return -1;
        PrecomputedTransactionData txdata;
        txdata.Init(tx, std::move(outs));
        if (!txdata.m_bip341_taproot_ready) return -1;  // SignatureHashSchnorr would assert
        ScriptExecutionData ed;
        ed.m_annex_init = true;
        ed.m_annex_present = annex != nullptr;
        if (annex) {
            std::vector<unsigned char> a(annex, annex + annexlen);
            ed.m_annex_hash = (CHashWriter(SER_GETHASH, 0) << a).GetSHA256();
        }
        if (sigversion == 1) {
            ed.m_tapleaf_hash_init = true;
            ed.m_tapleaf_hash = uint256(std::vector<unsigned char>(tapleaf32, tapleaf32 + 32));
            ed.m_codeseparator_pos_init = true;
            ed.m_codeseparator_pos = codesep_pos;
        }
        SchnorrCapturingChecker chk(&tx, nIn, 0, txdata);
        ScriptError serr = SCRIPT_ERR_OK;
        bool ok = chk.CheckSchnorrSignature(Span<const unsigned char>(sig, siglen),
                                            Span<const unsigned char>(pk32, 32),
                                            sigversion == 1 ? SigVersion::TAPSCRIPT : SigVersion::TAPROOT,
                                            ed, &serr);
        *serror = (int)serr;
        *hashed = chk.called ? 1 : 0;
        if (chk.called) memcpy(sighash32, chk.sighash.begin(), 32);
        return ok ? 1 : 0;
    } catch (const std::exception&) {
        return -1;
    }
}

// The reference's SignatureHash (interpreter.cpp:1576-1642) for one ECDSA check, obtained the way
// the interpreter obtains it: GenericTransactionSignatureChecker::CheckECDSASignature
// (:1656-1676) with a placeholder signature ending in `hashtype` and a placeholder 33-byte key,
// the sighash captured at VerifyECDSASignature.  sigversion 0 = BASE, 1 = WITNESS_V0.  Returns 1
// with sighash32 written, or -1 if the tx does not deserialize / nIn is out of range.
int ref_check_sighash(const unsigned char* txb, size_t txlen, unsigned int nIn,
                      const unsigned char* script, size_t scriptlen, unsigned int hashtype,
                      int64_t amount, int sigversion, unsigned char* sighash32) {
    try {
        ByteReader ss(txb, txlen);
        CTransaction tx(deserialize, ss);
        if (nIn >= tx.vin.size()) return -1;
        PrecomputedTransactionData txdata(tx);
        CapturingChecker chk(&tx, nIn, amount, txdata);
        std::vector<unsigned char> sig = {0x30, 0x06, 0x02, 0x01, 0x01, 0x02, 0x01, 0x01,
                                          (unsigned char)hashtype};
        std::vector<unsigned char> pub(33, 0x11);
        pub[0] = 0x02;
        chk.CheckECDSASignature(sig, pub, CScript(script, script + scriptlen),
                                sigversion == 1 ? SigVersion::WITNESS_V0 : SigVersion::BASE);
        if (chk.log.size() != 1) return -1;
        memcpy(sighash32, chk.log[0].sighash.begin(), 32);
        return 1;
    } catch (const std::exception&) {
        return -1;
    }
}

// ---- fixture generation helpers (NOT used by any parity check as a verdict source) ----
int ref_pubkey_create(const unsigned char* seckey32, int compressed, unsigned char* out,
                      size_t* outlen) {
    secp256k1_pubkey pk;
    if (!secp256k1_ec_pubkey_create(sign_ctx(), &pk, seckey32)) return 0;
    return secp256k1_ec_pubkey_serialize(sign_ctx(), out, outlen, &pk,
                                         compressed ? SECP256K1_EC_COMPRESSED
                                                    : SECP256K1_EC_UNCOMPRESSED);
}

int ref_sign(const unsigned char* seckey32, const unsigned char* msg32, unsigned char* der72,
             size_t* derlen) {
    secp256k1_ecdsa_signature sig;
    if (!secp256k1_ecdsa_sign(sign_ctx(), &sig, msg32, seckey32, nullptr, nullptr)) return 0;
    return secp256k1_ecdsa_signature_serialize_der(sign_ctx(), der72, derlen, &sig);
}

int ref_schnorr_sign(const unsigned char* seckey32, const unsigned char* msg32,
                     const unsigned char* aux32, unsigned char* sig64, unsigned char* xonly32) {
    secp256k1_keypair kp;
    if (!secp256k1_keypair_create(sign_ctx(), &kp, seckey32)) return 0;
    secp256k1_xonly_pubkey xpk;
    if (!secp256k1_keypair_xonly_pub(sign_ctx(), &xpk, nullptr, &kp)) return 0;
    if (!secp256k1_xonly_pubkey_serialize(sign_ctx(), xonly32, &xpk)) return 0;
    return secp256k1_schnorrsig_sign(sign_ctx(), sig64, msg32, &kp, nullptr, (void*)aux32);
}

// items are given as concatenated blobs with offset arrays (bitcoinconsensus_verify_script_
// with_amount per item, exactly what the crate's verify() calls).
double ref_bench_verify_script(int nthreads, long n, const unsigned char* spk_blob,
                               const long* spk_off, const unsigned char* tx_blob,
                               const long* tx_off, const int64_t* amounts,
                               const unsigned int* nin, unsigned int flags, int* ret) {
    return run_pool(nthreads, n, [=](long i) {
        bitcoinconsensus_error e;
        ret[i] = bitcoinconsensus_verify_script_with_amount(
            spk_blob + spk_off[i], (unsigned)(spk_off[i + 1] - spk_off[i]), amounts[i],
            tx_blob + tx_off[i], (unsigned)(tx_off[i + 1] - tx_off[i]), nin[i], flags, &e);
    });
}

// The same with the error code per item: ret[i] = result, err[i] = bitcoinconsensus_error
// (bulk script-level agreement checks).
double ref_bulk_verify_script(int nthreads, long n, const unsigned char* spk_blob,
                              const long* spk_off, const unsigned char* tx_blob, const long* tx_off,
                              const int64_t* amounts, const unsigned int* nin, unsigned int flags,
                              int* ret, int* err) {
    return run_pool(nthreads, n, [=](long i) {
        bitcoinconsensus_error e = bitcoinconsensus_ERR_OK;
        ret[i] = bitcoinconsensus_verify_script_with_amount(
            spk_blob + spk_off[i], (unsigned)(spk_off[i + 1] - spk_off[i]), amounts[i],
            tx_blob + tx_off[i], (unsigned)(tx_off[i + 1] - tx_off[i]), nin[i], flags, &e);
        err[i] = (int)e;
    });
}

// The same over an array of the engine's batch items (struct bcc_batch_item of the engine's
// include/bitcoinconsensus.h, restated here field by field): the bulk checker of agreement runs.
struct ref_batch_item {
    const unsigned char* spk;
    unsigned int spk_len;
    int64_t amount;
    const unsigned char* tx;
    unsigned int tx_len;
    unsigned int n_in;
};

double ref_bulk_verify_items(int nthreads, long n, const ref_batch_item* items, unsigned int flags,
                             int* ret, int* err) {
    return run_pool(nthreads, n, [=](long i) {
        bitcoinconsensus_error e = bitcoinconsensus_ERR_OK;
        const ref_batch_item& it = items[i];
        ret[i] = bitcoinconsensus_verify_script_with_amount(it.spk, it.spk_len, it.amount, it.tx,
                                                            it.tx_len, it.n_in, flags, &e);
        err[i] = (int)e;
    });
}

// The engine's bcc_taproot_check items (include/bcc_amd.h), restated field by field: the bulk
// checker / CPU baseline of the Taproot bench (CheckSchnorrSignature per item).
struct ref_taproot_item {
    const unsigned char* tx;
    unsigned int tx_len;
    const unsigned char* spent;
    unsigned int spent_len;
    unsigned int n_in;
    const unsigned char* sig;
    unsigned int sig_len;
    const unsigned char* pk32;
    int sigversion;
    const unsigned char* annex;
    unsigned int annex_len;
    const unsigned char* tapleaf32;
    uint32_t codesep_pos;
};

double ref_bulk_taproot(int nthreads, long n, const ref_taproot_item* items, int* ret, int* serr) {
    static const unsigned char zero32[32] = {0};
    return run_pool(nthreads, n, [=](long i) {
        const ref_taproot_item& it = items[i];
        unsigned char h[32];
        int hashed = 0;
        ret[i] = ref_taproot_check(it.tx, it.tx_len, it.spent, it.spent_len, it.n_in, it.sig,
                                   it.sig_len, it.pk32, it.sigversion, it.annex, it.annex_len,
                                   it.tapleaf32 ? it.tapleaf32 : zero32, it.codesep_pos, &serr[i],
                                   h, &hashed);
    });
}

// Tuple-level baseline: CPubKey::Verify over (pub, hash, sig) tuples. pub in 65-B slots with
// lengths, sig in 80-B slots with lengths.
double ref_bench_pubkey_verify(int nthreads, long n, const unsigned char* pub65, const int* publen,
                               const unsigned char* hash32, const unsigned char* sig80,
                               const int* siglen, int* ret) {
    return run_pool(nthreads, n, [=](long i) {
        ret[i] = ref_pubkey_verify(pub65 + 65 * i, (size_t)publen[i], hash32 + 32 * i,
                                   sig80 + 80 * i, (size_t)siglen[i]);
    });
}

// Tuple-level baseline / checker over blob inputs (uint64 offsets, n + 1 each): CPubKey::Verify.
double ref_bench_pubkey_verify_blob(int nthreads, long n, const unsigned char* pub_blob,
                                    const uint64_t* pub_off, const unsigned char* hash32,
                                    const unsigned char* sig_blob, const uint64_t* sig_off,
                                    unsigned char* ret) {
    return run_pool(nthreads, n, [=](long i) {
        ret[i] = (unsigned char)ref_pubkey_verify(
            pub_blob + pub_off[i], (size_t)(pub_off[i + 1] - pub_off[i]), hash32 + 32 * i,
            sig_blob + sig_off[i], (size_t)(sig_off[i + 1] - sig_off[i]));
    });
}

// BIP340 baseline / checker: secp256k1_xonly_pubkey_parse + secp256k1_schnorrsig_verify per row.
double ref_bench_schnorr_verify(int nthreads, long n, const unsigned char* sig64,
                                const unsigned char* msg32, const unsigned char* xonly32,
                                unsigned char* ret) {
    return run_pool(nthreads, n, [=](long i) {
        ret[i] = (unsigned char)ref_schnorr_verify(sig64 + 64 * i, msg32 + 32 * i,
                                                   xonly32 + 32 * i);
    });
}

}  // extern "C"
