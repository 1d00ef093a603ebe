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

/* ---- BIP341 / BIP342 (Taproot) signature checks ------------------------------------------------
 * Replaces GenericTransactionSignatureChecker::CheckSchnorrSignature per check
 * (depend/bitcoin/src/script/interpreter.cpp:1678-1704): SignatureHashSchnorr (:1491-1574) over
 * the tx's PrecomputedTransactionData initialised with its spent outputs (:1422-1472), then
 * XOnlyPubKey::VerifySchnorr (pubkey.cpp:176-182).  The signature hash (TapSighash tagged
 * SHA-256 and the tx's single-SHA-256 aux hashes) and the BIP340 verification run on the GPU.
 * The fields mirror the checker's inputs: the spending tx, the outputs it spends (one per input,
 * a serialized std::vector<CTxOut> as handed to PrecomputedTransactionData::Init), the input
 * index, the signature (64 bytes, or 65 with the hash_type), the 32-byte x-only key, the
 * sigversion and ScriptExecutionData's annex / tapleaf hash / OP_CODESEPARATOR position.
 * Adjacent items with the same tx and spent_outputs pointers share the per-tx hashes. */
#define BCC_SIGVERSION_TAPROOT 0   /* key path spend (SigVersion::TAPROOT) */
#define BCC_SIGVERSION_TAPSCRIPT 1 /* BIP342 script path (SigVersion::TAPSCRIPT) */
typedef struct bcc_taproot_check {
    const unsigned char* tx;            /* serialized spending tx, exactly tx_len bytes */
    unsigned int tx_len;
    const unsigned char* spent_outputs; /* serialized std::vector<CTxOut>, one per input */
    unsigned int spent_outputs_len;
    unsigned int n_in;
    const unsigned char* sig;           /* 64 or 65 bytes (anything else: SCHNORR_SIG_SIZE) */
    unsigned int sig_len;
    const unsigned char* pubkey32;      /* x-only key bytes */
    int sigversion;                     /* BCC_SIGVERSION_* */
    const unsigned char* annex;         /* the annex witness element incl. 0x50, NULL: none */
    unsigned int annex_len;
    const unsigned char* tapleaf_hash32; /* TAPSCRIPT only (execdata.m_tapleaf_hash) */
    uint32_t codeseparator_pos;         /* TAPSCRIPT only (0xFFFFFFFF: none executed) */
} bcc_taproot_check;
/* script_error.h:73-75 values written to serror_out */
#define BCC_SCRIPT_ERR_SCHNORR_SIG_SIZE 44
#define BCC_SCRIPT_ERR_SCHNORR_SIG_HASHTYPE 45
#define BCC_SCRIPT_ERR_SCHNORR_SIG 46
/* ret_out[i] = 1 (valid) or 0 (serror_out[i] = one of the three codes above), or -1 where the
 * reference checker cannot be built and asserts instead: the tx does not deserialize to exactly
 * tx_len bytes, the spent outputs do not parse or their count differs from the tx's inputs,
 * n_in >= inputs, or no witness-bearing input spends a 34-byte OP_1 script (the tx data would not
 * be BIP341-ready); serror_out[i] = 1 (SCRIPT_ERR_UNKNOWN_ERROR) then.  sighash_out (optional,
 * 32 bytes per item): the signature hash where one was computed, else zeros.  Synchronous on
 * `device`, or for device = -1 spread over the bcc_set_devices() GPUs.  Returns 0, or -1 on bad
 * arguments or a device failure (then no output is meaningful). */
int bcc_taproot_verify_batch(const bcc_taproot_check* items, size_t n, int* ret_out,
                             int* serror_out, unsigned char* sighash_out, int device);

/* ---- tuple level with the CPubKey front end ---------------------------------------------------
 * verdict[i] = CPubKey(pub_i).Verify(msg_i, sig_i) (depend/bitcoin/src/pubkey.cpp:191-207) for n
 * tuples: pub_i = pub_blob[pub_off[i] .. pub_off[i+1]) (any length; the CPubKey length filter,
 * pubkey.h:58-94, applies), sig_i = sig_blob[sig_off[i] .. sig_off[i+1]) = DER without the
 * hashtype byte, parsed laxly (pubkey.cpp:28-168).  The blobs go to the GPU as they are and the
 * length filter and lax DER run there (K_der, csrc/der.hip), in pipelined rounds of 256k doubling
 * to 2M tuples; small rounds run on the host lane code.  Synchronous on `device`, or, for
 * device = -1, sharded in contiguous equal ranges over the bcc_set_devices() GPUs.  0, or -1 for
 * null arrays, offsets that are not non-decreasing (pub_off[i + 1] < pub_off[i] or
 * sig_off[i + 1] < sig_off[i] for any i: nothing is verified, so no verdict depends on how the call
 * is cut into rounds), or a device error. */
int bcc_pubkey_verify_batch(const uint8_t* pub_blob, const uint64_t* pub_off,
                            const uint8_t* msg32, const uint8_t* sig_blob,
                            const uint64_t* sig_off, uint8_t* verdict, size_t n, int device);

/* ---- engine configuration / statistics ---------------------------------------------------- */
/* Hash of the sources this library was built from (rust-bitcoinconsensus_amd/source_hash.py):
 * callers can check that the library they loaded matches the tree they test. */
const char* bcc_source_hash(void);

/* Device used by the bitcoinconsensus_* entry points of the calling process (default 0, or the
 * BCC_DEVICE environment variable). */
int bcc_set_device(int device);

/* Node sharding: spread every device round of bitcoinconsensus_verify_batch, and
 * bcc_pubkey_verify_batch(..., device = -1), over these GPUs (default: the single device above,
 * or BCC_DEVICES="0,1,2,..." in the environment; n = 0 restores the default).  A round is cut
 * into contiguous groups of whole transactions with about equal signature counts, one per GPU;
 * the groups run concurrently, each GPU from its own persistent host worker thread (its own HIP
 * stream, device arena and kernel scratch), and the verdicts are gathered on the host.  Results
 * never depend on the device set.  Returns 0, or -1 for a negative device id. */
int bcc_set_devices(const int* devices, int n);
/* Writes up to cap configured device ids to out; returns how many there are. */
int bcc_get_devices(int* out, int cap);

/* Lanes per signature-kernel launch (0 = default: 4M, or the BCC_CHUNK environment variable).
 * Bounds the per-caller device scratch (900 B per lane); results do not depend on it. */
int bcc_set_chunk_lanes(size_t lanes);

/* bitcoinconsensus_verify_batch pipelines a batch of at least two chunks: it is cut into chunks of
 * about `items` inputs (whole transactions), and each chunk's device round runs on a worker thread
 * while the host deserializes and interprets the next chunk.  Default 500000 (or the
 * BCC_PIPELINE_CHUNK environment variable); 0 disables it.  Results never depend on it. */
int bcc_set_pipeline_chunk(size_t items);
/* Items of a pipelined batch's last chunk (its device round is the one no host pass hides):
 * 0 (default, or BCC_PIPELINE_TAIL) keeps the remainder; results never depend on it. */
int bcc_set_pipeline_tail(size_t items);
/* Host shards per worker thread of a long bitcoinconsensus_verify_batch pass (default 1, or
 * BCC_LONG_SHARDS_PER_WORKER): with k > 1 the k x workers shards are dealt dynamically.  Results
 * never depend on it.  Returns 0, or -1 for k outside 1..64. */
int bcc_set_long_shards_per_worker(unsigned k);
/* bitcoinconsensus_verify_batch's first interpreter pass runs inside the parse pass, block by
 * block per host shard, while each item's transaction is still in cache (default 1, or
 * BCC_FUSED_PASS; 0: two passes).  Calls with early Q halves keep two passes.  Results never
 * depend on it.  Returns 0. */
int bcc_set_fused_pass(int on);
/* A device round's tuple rows, raw transactions and sighash blobs are written by the host pass into
 * page-locked memory and go to HBM from there, one copy per host shard and array; staging copies
 * only the records whose offsets it rebases (default 1, or BCC_DIRECT_UPLOAD; 0: every array is
 * copied into one pinned image first).  Results never depend on it.  Returns 0. */
int bcc_set_direct_upload(int on);
/* With the direct upload, each host shard of a pipelined bitcoinconsensus_verify_batch chunk sends
 * its tuple rows to the GPU as soon as the pass has finished it, and the chunk's device round
 * gathers them in HBM instead of uploading them (default 1, or BCC_PRE_UPLOAD).  Results never
 * depend on it.  Returns 0. */
int bcc_set_pre_upload(int on);

/* Legacy signature checks whose serial SHA-256 chain is longer than `blocks` 64-byte blocks (the
 * preimages of many-input transactions) are hashed on the host CPU instead of in one GPU lane each,
 * while the device round's message-independent kernels run (BCC_HOST_CHAIN_BLOCKS; default 160,
 * below the Q ladder's latency in GPU-lane blocks; 0: every legacy chain on the GPU).  A long
 * transaction template carries its SHA-256 midstates, so a check's chain counts only the blocks
 * from its own input's script on (host and GPU start from the midstate alike).  Single-GPU
 * rounds only, at most 2^19 blocks per interpreter pass.  BIP143 checks of a tx whose
 * per-tx chains (hashPrevouts / hashSequence / hashOutputs) exceed BCC_HOST_BIP143_BLOCKS (default
 * 32) blocks are hashed on the host (linear in the tx).  Results never depend on either. */
int bcc_set_host_chain_blocks(unsigned blocks);
/* The BIP143 threshold above (BCC_HOST_BIP143_BLOCKS; default 32; 0: every BIP143 chain on the GPU). */
int bcc_set_host_bip143_blocks(unsigned blocks);

/* Early Q halves (BCC_EARLY_Q; default 1): a verify_batch call that goes to one GPU as one chunk
 * (at most 2^18 inputs) pre-extracts the (key, signature) pairs of its standard spends after
 * deserialization and runs their key half and Q ladder on the GPU while the host interprets; the
 * interpreter's deferred checks with the same key and signature bytes reuse them.  0 disables it.
 * Results never depend on it. */
int bcc_set_early_q(int on);

/* Key-hash spends (P2WPKH, and P2PKH scriptPubKeys): on an input's first interpreter run the
 * HASH160(pubkey) == program comparison of OP_EQUALVERIFY is checked on the device beside the
 * signature (the row's verdict = signature valid AND hash equal); a false verdict re-runs the
 * input on the host with the comparison done there, so the error codes are the reference's.
 * on = 0: the host hashes every P2WPKH key before the run (BCC_DEVICE_KEY_HASH; default 1).
 * Results never depend on it. */
int bcc_set_device_key_hash(int on);

/* Host worker threads of a batch pass (verify_batch interpreter shards, tuple / Taproot front
 * ends, host-verified rounds).  0 restores the default: BCC_HOST_THREADS, else the CPUs of the
 * affinity mask, or the cgroup CPU quota when that is smaller, at most 64.  Results never
 * depend on it. */
int bcc_set_host_threads(unsigned n);
unsigned bcc_get_host_threads(void);
/* CPUs this process can keep busy: min(affinity mask, cgroup CPU quota). */
unsigned bcc_cpu_share(void);

/* bitcoinconsensus_verify_batch keeps its host-side state (items, parsed transactions, job
 * buffers) with the calling thread for reuse by its next call; batches above 4M items release it
 * on return.  bcc_taproot_verify_batch keeps its job buffers the same way, and every entry point
 * keeps a device batch (HBM arena, pinned staging image, streams, kernel scratch) per (thread,
 * GPU).  This releases the calling thread's state, and the state the library's own worker threads
 * keep (the per-GPU workers of a bcc_set_devices() list and the pipeline worker run rounds for
 * their callers), now.
 * Threads: with one device and no pipelining a call runs on the calling thread with that
 * thread's own device state, so concurrent callers share nothing.  With several devices
 * configured, or pipelining on, device rounds run on one shared worker thread per GPU: the results
 * are the same, but concurrent callers' rounds queue on those workers. */
void bcc_release_thread_state(void);

typedef struct bcc_batch_stats {
    size_t items, tuples, rounds, preimages, aux_messages, host_rejected;
    double host_seconds, gpu_seconds;
    /* breakdown: host deserialize + pre-checks, interpreter passes (preimage building
     * included), merging the per-thread rounds, host -> HBM staging (part of gpu_seconds) */
    double prepare_seconds, interpret_seconds, merge_seconds, stage_seconds;
    double total_seconds; /* the whole call, teardown included */
    size_t device_retries; /* device rounds that failed once and were re-run on a fresh batch */
    size_t devices;        /* GPUs a device round was spread over (max over the call's rounds) */
    size_t host_rounds;    /* rounds (or device groups) verified on the host CPU: small rounds
                            * (bcc_set_host_small_round) and device-failure fallbacks */
    size_t host_hashed;    /* deferred checks whose sighash the host computed (SHA chains longer
                            * than bcc_set_host_chain_blocks) */
    /* more of the host pass: shard / run lists, stitching verdicts into items, writing ret / err,
     * the host-hashed long chains */
    double shard_seconds, stitch_seconds, finish_seconds, host_jobs_seconds;
    /* the deserialization pass per worker, max over workers (summed over chunks): dispatch -> start
     * lag, tx parsing + pre-checks, the batched HASH160 of P2WPKH keys */
    double prepare_lag_seconds, prepare_parse_seconds, prepare_hash_seconds;
    /* key-hash conditions (HASH160(pubkey) == program) checked on the device beside their
     * signature (bcc_set_device_key_hash) */
    size_t device_key_hashes;
    /* interpreter passes per shard: the slowest shard and the mean (summed over passes): their
     * ratio is the passes' load imbalance */
    double interpret_shard_max_seconds, interpret_shard_mean_seconds;
    /* CPU time of the whole process (every thread) during the call, and during the caller's waits
     * for device rounds: under a CFS quota the first bounds back-to-back calls */
    double process_cpu_seconds, process_cpu_in_gpu_wait_seconds;
    /* early Q halves (bcc_set_early_q): pre-extracted rows whose key half and Q ladder ran on the
     * GPU during the host pass, the deferred rows mapped to them, and the extraction + launch time */
    size_t early_rows, early_mapped;
    double early_seconds;
    /* ... and the mapped rows whose legacy sighash came from the early set too (early sighashes:
     * long-template SIGHASH_ALL jobs hashed during the host pass, the round's copy skipped) */
    size_t early_msgs;
} bcc_batch_stats;
/* Statistics of the calling thread's last bitcoinconsensus_verify_batch / verify call. */
void bcc_last_batch_stats(bcc_batch_stats* out);

/* ---- host verification: the engine's own code on the CPU ------------------------------------
 * A device round (sighash jobs + ECDSA tuples) can be evaluated on the host with the engine's own
 * preimage builders, host SHA-256 and the kernels' lane code compiled for the CPU
 * (csrc/host/host_verify.cpp); the verdicts are the same.
 *
 * Device failure policy.  A failed device round is retried once on a fresh device batch when the
 * HIP error is transient (out of memory, not ready); a sticky error (launch failure, illegal
 * address, no device, ...) leaves the HIP context unusable, so it is not retried.  Then:
 *   BCC_DEVICE_FAILURE_HOST  (default; BCC_DEVICE_FAILURE=host) the round is verified on the host
 *                            CPU (logged on stderr, counted by bcc_host_fallback_rounds) and every
 *                            entry point returns its normal, exact result;
 *   BCC_DEVICE_FAILURE_ERROR (BCC_DEVICE_FAILURE=error) bitcoinconsensus_verify_batch returns -1
 *                            (unfinished items: BCC_ERR_DEVICE_FAILURE) and the single-item ABI
 *                            aborts, as there is no verdict (see bitcoinconsensus.h). */
#define BCC_DEVICE_FAILURE_HOST 0
#define BCC_DEVICE_FAILURE_ERROR 1
int bcc_set_device_failure_policy(int policy);
/* Device rounds of at most `tuples` signature checks are verified on the host CPU with the
 * engine's own lane code instead of the GPU (default BCC_HOST_SMALL_ROUND_DEFAULT, or the
 * BCC_HOST_SMALL_ROUND environment variable; 0: every round on the GPU).  One lane of the GPU
 * ladder is a single wave issuing a few hundred thousand dependent instructions, so a lone
 * verify() costs ~1.6 ms as a GPU round and ~0.1 ms on the host. */
#define BCC_HOST_SMALL_ROUND_DEFAULT 16
int bcc_set_host_small_round(size_t tuples);
/* Device rounds (or per-GPU groups) verified on the host after a device failure, process-wide. */
size_t bcc_host_fallback_rounds(void);
/* mi_ecdsa_verify_tuples' contract on the host CPU (threads >= 1). */
int bcc_host_verify_tuples(const uint8_t* pub65, const uint8_t* msg32, const uint8_t* r32,
                           const uint8_t* s32, uint8_t* verdict, size_t n, unsigned threads);

/* Fault injection (tests): the next `rounds` device rounds of any thread fail as if the HIP
 * runtime had returned a transient error (hipErrorOutOfMemory), without touching the GPU (also:
 * BCC_FAULT_INJECT=rounds in the environment at load time); _code injects the given HIP error
 * (e.g. 719, hipErrorLaunchFailure: sticky, never retried). */
void bcc_debug_fail_device_rounds(int rounds);
void bcc_debug_fail_device_rounds_code(int rounds, int hip_error);
/* Test hook: signature-kernel scratch requests above `lanes` lanes fail as out of memory (0: no
 * cap).  The kernels then run in the largest chunk that fits (halving from the request, at least
 * 64k lanes) instead of failing the round. */
void bcc_debug_scratch_cap_lanes(size_t lanes);

#ifdef __cplusplus
}
#endif

#endif
