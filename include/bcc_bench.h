/* bcc_bench.h — C ABI of librbc_bench.so: synthetic workloads, signature generators, the
 * integer-ALU microbenchmark and the field self-test.  NOT part of the product: bench.py, the
 * tests and the tools drive the product library (librbc_amd.so, include/bcc_amd.h and
 * include/bitcoinconsensus.h) through these.  librbc_bench.so links librbc_amd.so and stages its
 * inputs with the product's own host passes (the first interpreter round) and device batches.
 */
#ifndef BCC_BENCH_H
#define BCC_BENCH_H

#include <stddef.h>
#include <stdint.h>

#include "bcc_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- synthetic tuple sets (configs C4 / C5; bench.py / tests), staged in HBM ---------------- */
typedef struct bcc_tupleset bcc_tupleset;
/* C4: n (pub, msg32, DER sig) tuples from `seed`, 90 % valid, 10 % over 18 adversarial classes
 * (bit-flipped r / s / msg, high-S, r or s >= n, r or s = 0, over-long and zero-padded r,
 * compressed x without a square root, x >= p, 04 with a wrong y, 04, hybrid 06/07 with good and
 * bad parity, bad header, wrong key).  The staged rows are those bcc_pubkey_verify_batch builds. */
bcc_tupleset* bcc_tupleset_c4(size_t n, uint64_t seed, int device);
/* Tuples [first, first + n) of the global C4 set of `total` tuples from `seed` (the node batch
 * partitioned by rank: every tuple depends only on (seed, its global index, total)). */
bcc_tupleset* bcc_tupleset_c4_range(size_t n, uint64_t seed, size_t first, size_t total,
                                    int device);
/* C5: n BIP340 rows, fresh GPU-signed from `seed`, with the nvec caller vectors (sig64, msg32,
 * xonly32, expected verdict) at rows i with i % 1024 == 1 + j. */
bcc_tupleset* bcc_tupleset_c5(size_t n, uint64_t seed, const uint8_t* vec_sig64,
                              const uint8_t* vec_msg32, const uint8_t* vec_xonly32,
                              const uint8_t* vec_expect, size_t nvec, int device);
/* Rows [first, first + n) of the global C5 set (vectors tiled by global index). */
bcc_tupleset* bcc_tupleset_c5_range(size_t n, uint64_t seed, size_t first,
                                    const uint8_t* vec_sig64, const uint8_t* vec_msg32,
                                    const uint8_t* vec_xonly32, const uint8_t* vec_expect,
                                    size_t nvec, int device);
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

/* ---- synthetic workloads (bench.py / tests): built and staged on the device ---------------- */
typedef struct bcc_workload bcc_workload;

/* C2: n synthetic P2WPKH spends (1-in/1-out v2 txs, BIP143 SIGHASH_ALL, low-S DER), keys,
 * nonces and amounts derived from `seed`.  Keys and signatures are produced by
 * the engine's own GPU kernels; txs / sighash jobs are staged in HBM. */
bcc_workload* bcc_workload_p2wpkh(size_t n, uint64_t seed, int device);
/* Spends [first, first + n) of the global C2 set from `seed` (rank partitions of one set). */
bcc_workload* bcc_workload_p2wpkh_range(size_t n, uint64_t seed, size_t first, int device);
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
/* C2-style staging of ANY caller items (copied): the engine's first interpreter round under
 * `flags`, staged in HBM exactly as for the synthetic workloads (parity tests of the benchmarked
 * staged path on mutated inputs). */
bcc_workload* bcc_workload_from_items(const bcc_batch_item* items, size_t n, unsigned flags,
                                      int device);
/* Copy back the verdicts of the staged tuple rows: one byte per tuple row (bcc_workload_shape's
 * `tuples`; a block workload's multisig inputs stage several rows per item).  `cap` is the size of
 * `out` in bytes.  Returns 0, -1 for a NULL workload / buffer, BCC_BENCH_ERR_CAPACITY when cap is
 * smaller than the row count (nothing written), or a HIP error. */
#define BCC_BENCH_ERR_CAPACITY (-2)
int bcc_workload_verdicts(bcc_workload* w, uint8_t* out, size_t cap);
/* Mutated copies of a workload's items for agreement runs (see workload.cpp): kinds[i] = 0 for an
 * untouched item, else 1 + the mutation (bit flip anywhere in the tx / in its back half, amount
 * +-1, spent-script bit flip, truncated tx, nIn out of range).  Valid while the set lives. */
typedef struct bcc_itemset bcc_itemset;
bcc_itemset* bcc_workload_mutate(const bcc_workload* w, double rate, uint64_t seed,
                                 uint8_t* kinds);
const bcc_batch_item* bcc_itemset_items(const bcc_itemset* m, size_t* n);
void bcc_itemset_free(bcc_itemset* m);
/* item index of every staged tuple row (uint32 per tuple); `cap` in entries.  Returns 0, -1 for a
 * NULL workload / buffer, BCC_BENCH_ERR_CAPACITY when cap < tuples (nothing written). */
int bcc_workload_tuple_items(const bcc_workload* w, uint32_t* out, size_t cap);
/* the sighash (msg32) rows of the last run, 32 bytes per tuple (synchronous); `cap` in bytes.
 * Returns 0, -1, BCC_BENCH_ERR_CAPACITY when cap < 32 x tuples (nothing written), or a HIP error. */
int bcc_workload_msgs(bcc_workload* w, uint8_t* out, size_t cap);
/* algorithmic work of one run: bytes hashed + written by the sighash stage, tuples verified */
/* algorithmic bytes of one sighash-stage run over the staged batch (DeviceBatch::sighash_bytes) */
size_t bcc_workload_sighash_bytes(const bcc_workload* w);
void bcc_workload_shape(const bcc_workload* w, size_t* tuples, size_t* sighash_blocks,
                        size_t* aux_blocks, size_t* preimages, size_t* aux_messages);
/* export item i as (spk, amount, tx) for CPU-baseline / parity checks: returns tx length and
 * copies up to cap bytes; *spk_len <= 64 */
size_t bcc_workload_item(const bcc_workload* w, size_t i, uint8_t* spk, size_t* spk_len,
                         int64_t* amount, uint8_t* tx, size_t cap);

/* ---- the GPU sighash stage alone (tests) ----------------------------------------------------
 * One signature check's SignatureHash inputs (interpreter.cpp:1576-1642): the spending tx, the
 * input index, the scriptCode as the checker receives it (OP_CODESEPARATORs still in for legacy:
 * the serializer drops them), the full 32-bit hash type, the amount (BIP143) and the SigVersion
 * (0 BASE, 1 WITNESS_V0). */
typedef struct bcc_sighash_check {
    const uint8_t* tx;
    size_t tx_len;
    const uint8_t* script_code;
    size_t script_code_len;
    unsigned int n_in;
    int32_t hashtype;
    int64_t amount;
    int sigversion;
} bcc_sighash_check;
/* Builds each check's device job exactly as the batch engine's deferring checker does and runs
 * only the sighash kernels on `device`; msg32_out receives the n message rows the ECDSA kernels
 * would read (the SHA-256d sighash as raw uint256 bytes; uint256 ONE for the SIGHASH_SINGLE bug).
 * Returns 0, -1 for a tx that does not parse / a bad index or sigversion, or a HIP error. */
int bcc_debug_sighash(const bcc_sighash_check* checks, size_t n, uint8_t* msg32_out, int device);

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
/* Sustained form (the roofline peak): waves_per_simd waves of op per SIMD, launches of about
 * target_ms back to back for warm_s seconds, then reps timed launches; median lane-instructions/s,
 * median in-kernel clock (GHz, s_memtime / s_memrealtime stamps per wave) and launch time. */
int mi_microbench_sustained(int op, int waves_per_simd, double target_ms, double warm_s, int reps,
                            double* rate, double* clock_ghz, double* ms);

/* Per-primitive cost (tests of the ladder's cost model): prim 0 fe_mul, 1 fe_sqr, 2 fe_add,
 * 3 fe_sub, 4 fe_shl<1>, 5 gej_double, 6 gej_add_zinv (mixed), looped iters times per lane at
 * 4 waves per SIMD; *cycles = median SIMD-clock cycles per primitive per wave. */
int mi_primbench(int prim, int iters, int warm, double* cycles, double* ms);

/* ---- field self-test (tests only): one device Fp operation over n operand pairs ------------
 * a, b, out: n x 8 little-endian u32 limbs.  op: 0 add, 1 sub, 2 mul, 3 sqr, 4/5/6 shift by
 * 1/2/3, 7 neg, 8 is_zero (out[0]), 9 normalize, 10 fe_inv (mod p), 11 sc_inv (mod n, a < n).
 * Results are weak (< 2^256) except 8-11. */
int mi_fe_selftest(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n);

#ifdef __cplusplus
}
#endif

#endif
