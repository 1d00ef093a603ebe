/* bcc_amd.h — engine-level C ABI of librbc_amd.so below the drop-in interface.
 *
 * These are the entry points the reference's FFI would bind for the signature hot path once the
 * interpreter defers its checks ("New ABI to add"), plus the device-pointer and
 * workload entry points bench.py drives.  No torch / HIP types appear in any signature: device
 * buffers and streams are passed as plain pointers.
 */
#ifndef BCC_AMD_H
#define BCC_AMD_H

#include <stddef.h>
#include <stdint.h>

#include "bitcoinconsensus.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- tuple level: the deferred CHECKSIG queue flushed to the GPU ---------------------------
 * Replaces the per-signature call CPubKey::Verify -> secp256k1_ecdsa_verify
 * (depend/bitcoin/src/pubkey.cpp:191-207, secp256k1/src/secp256k1.c:423-438).
 * pub65[i] = header byte || x || y (y ignored for 02/03; header 0 marks a key the caller's
 * CPubKey length filter already rejected); msg32 = raw sighash bytes; r32/s32 = big-endian
 * scalars after lax-DER parsing (both zero on overflow).  verdict[i] = 1 iff valid. */
int mi_ecdsa_verify_tuples(const uint8_t* pub65, const uint8_t* msg32, const uint8_t* r32,
                           const uint8_t* s32, uint8_t* verdict, size_t n, int device);

/* Same with all buffers device-resident (separate tag / x / y / r / s / m rows), launched on
 * `stream` (a hipStream_t or NULL).  Asynchronous. */
int mi_ecdsa_verify_device(const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                           const uint8_t* d_r, const uint8_t* d_s, const uint8_t* d_m,
                           uint8_t* d_verdict, size_t n, void* stream);

/* ---- BIP340 Schnorr (config C5) -------------------------------------------------------------
 * Replaces secp256k1_xonly_pubkey_parse + secp256k1_schnorrsig_verify per signature
 * (secp256k1/src/modules/extrakeys/main_impl.h:21-39, modules/schnorrsig/main_impl.h:190-237),
 * as bound by Core's XOnlyPubKey::VerifySchnorr (depend/bitcoin/src/pubkey.cpp:176-182).
 * Row i: sig64 = r.x || s, msg32, xonly32 = the key's 32 serialized bytes (a key that does not
 * parse verifies false).  verdict[i] = 1 iff valid. */
int mi_schnorr_verify_tuples(const uint8_t* sig64, const uint8_t* msg32, const uint8_t* xonly32,
                             uint8_t* verdict, size_t n, int device);
/* Same with device-resident rows, launched on `stream`.  Asynchronous. */
int mi_schnorr_verify_device(const uint8_t* d_sig64, const uint8_t* d_msg32,
                             const uint8_t* d_xonly32, uint8_t* d_verdict, size_t n,
                             void* stream);

/* ---- tuple level with the CPubKey front end ---------------------------------------------------
 * verdict[i] = CPubKey(pub_i).Verify(msg_i, sig_i) (depend/bitcoin/src/pubkey.cpp:191-207) for n
 * tuples: pub_i = pub_blob[pub_off[i] .. pub_off[i+1]) (any length; the CPubKey length filter,
 * pubkey.h:58-94, applies), sig_i = sig_blob[sig_off[i] .. sig_off[i+1]) = DER without the
 * hashtype byte, parsed laxly (pubkey.cpp:28-168).  Synchronous on `device`.  0 or an error. */
int bcc_pubkey_verify_batch(const uint8_t* pub_blob, const uint64_t* pub_off,
                            const uint8_t* msg32, const uint8_t* sig_blob,
                            const uint64_t* sig_off, uint8_t* verdict, size_t n, int device);

/* ---- synthetic tuple sets (configs C4 / C5; bench.py / tests), staged in HBM ---------------- */
typedef struct bcc_tupleset bcc_tupleset;
/* C4: n (pub, msg32, DER sig) tuples from `seed`, 90 % valid, 10 % over 18 adversarial classes
 * (bit-flipped r / s / msg, high-S, r or s >= n, r or s = 0, over-long and zero-padded r,
 * compressed x without a square root, x >= p, 04 with a wrong y, 04, hybrid 06/07 with good and
 * bad parity, bad header, wrong key).  The staged rows are those bcc_pubkey_verify_batch builds. */
bcc_tupleset* bcc_tupleset_c4(size_t n, uint64_t seed, int device);
/* C5: n BIP340 rows, fresh GPU-signed from `seed`, with the nvec caller vectors (sig64, msg32,
 * xonly32, expected verdict) at rows i with i % 1024 == 1 + j. */
bcc_tupleset* bcc_tupleset_c5(size_t n, uint64_t seed, const uint8_t* vec_sig64,
                              const uint8_t* vec_msg32, const uint8_t* vec_xonly32,
                              const uint8_t* vec_expect, size_t nvec, int device);
void bcc_tupleset_free(bcc_tupleset* ts);
size_t bcc_tupleset_size(const bcc_tupleset* ts);
/* launch the verify kernels over the resident rows on `stream` (asynchronous) */
int bcc_tupleset_run(bcc_tupleset* ts, void* stream);
/* copy back the n verdicts of the last run (synchronous) */
int bcc_tupleset_verdicts(bcc_tupleset* ts, uint8_t* out);
/* host copies of the inputs (valid while ts lives); cls = generator class (0 = plain valid),
 * expect = verdict by construction.  C4 fills pub / sig, C5 fills sig64 / xonly32. */
typedef struct bcc_tupleset_host {
    size_t n;
    const uint8_t *pub_blob, *sig_blob, *msg32, *sig64, *xonly32, *cls, *expect;
    const uint64_t *pub_off, *sig_off;
} bcc_tupleset_host;
void bcc_tupleset_view(const bcc_tupleset* ts, bcc_tupleset_host* v);

/* ---- engine configuration / statistics ---------------------------------------------------- */
/* Device used by the bitcoinconsensus_* entry points of the calling process (default 0, or the
 * BCC_DEVICE environment variable). */
int bcc_set_device(int device);

/* Lanes per signature-kernel launch (0 = default: 4M, or the BCC_CHUNK environment variable).
 * Bounds the per-caller device scratch (900 B per lane); results do not depend on it. */
int bcc_set_chunk_lanes(size_t lanes);

/* bitcoinconsensus_verify_batch keeps its host-side state (items, parsed transactions, job
 * buffers) with the calling thread for reuse by its next call; batches above 4M items release it
 * on return.  This releases the calling thread's state now. */
void bcc_release_thread_state(void);

typedef struct bcc_batch_stats {
    size_t items, tuples, rounds, preimages, aux_messages, host_rejected;
    double host_seconds, gpu_seconds;
    /* breakdown: host deserialize + pre-checks, interpreter passes (preimage building
     * included), merging the per-thread rounds, host -> HBM staging (part of gpu_seconds) */
    double prepare_seconds, interpret_seconds, merge_seconds, stage_seconds;
    double total_seconds; /* the whole call, teardown included */
} bcc_batch_stats;
/* Statistics of the calling thread's last bitcoinconsensus_verify_batch / verify call. */
void bcc_last_batch_stats(bcc_batch_stats* out);

/* ---- synthetic workloads (bench.py / tests): built and staged on the device ---------------- */
typedef struct bcc_workload bcc_workload;

/* C2: n synthetic P2WPKH spends (1-in/1-out v2 txs, BIP143 SIGHASH_ALL, low-S DER), keys,
 * nonces and amounts derived from `seed`.  Keys and signatures are produced by
 * the engine's own GPU kernels; txs / sighash jobs are staged in HBM. */
bcc_workload* bcc_workload_p2wpkh(size_t n, uint64_t seed, int device);
/* C3: block replay.  ntx transactions with tx_nin[j] inputs / tx_nout[j] outputs (the histogram
 * of the reference's bench/data/block413567.raw), inputs 60 % P2PKH / 30 % P2WPKH / 10 % P2SH
 * 2-of-3 multisig, re-signed with synthetic keys from `seed`.  One item per
 * input, in transaction order. */
bcc_workload* bcc_workload_block(const uint32_t* tx_nin, const uint32_t* tx_nout, size_t ntx,
                                 uint64_t seed, int device);
void bcc_workload_free(bcc_workload* w);
/* the workload's items (valid while w lives), e.g. for bitcoinconsensus_verify_batch */
const bcc_batch_item* bcc_workload_items(const bcc_workload* w, size_t* n);
size_t bcc_workload_size(const bcc_workload* w);
/* launch the full hot path (sighash kernels + ECDSA kernel) on the staged inputs */
int bcc_workload_run(bcc_workload* w, void* stream);
int bcc_workload_run_sighash(bcc_workload* w, void* stream);
int bcc_workload_run_ecdsa(bcc_workload* w, void* stream);
/* copy back verdicts (n bytes) */
int bcc_workload_verdicts(bcc_workload* w, uint8_t* out);
/* algorithmic work of one run: bytes hashed + written by the sighash stage, tuples verified */
void bcc_workload_shape(const bcc_workload* w, size_t* tuples, size_t* sighash_blocks,
                        size_t* aux_blocks, size_t* preimages, size_t* aux_messages);
/* export item i as (spk, amount, tx) for CPU-baseline / parity checks: returns tx length and
 * copies up to cap bytes; *spk_len <= 64 */
size_t bcc_workload_item(const bcc_workload* w, size_t i, uint8_t* spk, size_t* spk_len,
                         int64_t* amount, uint8_t* tx, size_t cap);

/* ---- generator kernels (synthetic inputs; not on the verification path) -------------------- */
int mi_gen_pubkeys(const uint8_t* d32, size_t n, uint8_t* x32, uint8_t* y32, uint8_t* ok,
                   int device);
int mi_gen_sign(const uint8_t* d32, const uint8_t* m32, const uint8_t* k32, size_t n,
                uint8_t* r32, uint8_t* s32, uint8_t* ok, int device);
/* BIP340 sig64 (nonce k given) + the x-only key of d, for n (d, m, k) rows. */
int mi_gen_schnorr_sign(const uint8_t* d32, const uint8_t* m32, const uint8_t* k32, size_t n,
                        uint8_t* sig64, uint8_t* xonly32, uint8_t* ok, int device);

/* ---- integer-ALU microbenchmark (the roofline peak) ---------------------------------------- */
int mi_microbench(int op, int iters, double* rate);

/* ---- field self-test (tests only): one device Fp operation over n operand pairs ------------
 * a, b, out: n x 8 little-endian u32 limbs.  op: 0 add, 1 sub, 2 mul, 3 sqr, 4/5/6 shift by
 * 1/2/3, 7 neg, 8 is_zero (out[0]), 9 normalize.  Results are weak (< 2^256) except 8, 9. */
int mi_fe_selftest(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n);

#ifdef __cplusplus
}
#endif

#endif
