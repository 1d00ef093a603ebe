/* bitcoinconsensus.h — drop-in C ABI of the MI355X engine (librbc_amd.so).
 *
 * Same symbols, signatures, return convention and error ordering as libbitcoinconsensus v0.21,
 * which rust-bitcoinconsensus binds in src/lib.rs:145-161:
 *
 *   bitcoinconsensus_verify_script_with_amount  replaces depend/bitcoin/src/script/bitcoinconsensus.h:200-202
 *                                               (bitcoinconsensus.cpp:104-110), bound at src/lib.rs:151-160
 *   bitcoinconsensus_verify_script              replaces bitcoinconsensus.h:196-198 (bitcoinconsensus.cpp:113-123)
 *   bitcoinconsensus_version                    replaces bitcoinconsensus.h:204 (bitcoinconsensus.cpp:125-129),
 *                                               bound at src/lib.rs:148
 *
 * plus the north-star extension
 *
 *   bitcoinconsensus_verify_batch               N independent (script, amount, tx, nIn) checks; per-item
 *                                               results equal N calls of ..._with_amount
 *
 * Return convention: 1 = valid, 0 = invalid or error; *err is written only when err != NULL.
 * Check order: flags -> deserialize -> nIn -> size -> (ERR_OK) -> script.
 * Where signature checks run: a round of more than BCC_HOST_SMALL_ROUND_DEFAULT (16) checks is
 * verified on the GPU (HIP, gfx950).  Smaller rounds (a lone call of ..._with_amount, tiny batches)
 * run on the host CPU with the kernels' own lane arithmetic compiled for the host, because one GPU
 * lane's ladder latency exceeds the whole host check (bcc_amd.h: bcc_set_host_small_round; 0 puts
 * every round on the GPU).  Rounds the GPU could not deliver go to the host as described under
 * "Device failure" below.  Either way the verdicts are the reference's.
 * Thread safety: reentrant.  Each calling thread gets its own HIP stream, device arena, pinned
 * staging buffer and kernel scratch per device (created on its first call, reused afterwards), so
 * concurrent callers never share mutable device state; the only shared state is the read-only
 * G table per device, built once under a lock.
 * Device failure: a failed device round is retried once on a fresh batch when the error is
 * transient.  If the device still cannot deliver, the round is verified on the host CPU with the
 * engine's own code (bcc_amd.h: BCC_DEVICE_FAILURE_HOST, the default) and every entry point
 * returns its exact result.  Under BCC_DEVICE_FAILURE_ERROR there is no verdict:
 * bitcoinconsensus_verify_script[_with_amount] abort() the process (returning 0 would report a
 * consensus failure for a transaction that may be valid) and bitcoinconsensus_verify_batch returns
 * -1 instead (see below).
 */
#ifndef BCC_AMD_BITCOINCONSENSUS_H
#define BCC_AMD_BITCOINCONSENSUS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BITCOINCONSENSUS_API_VER 1

typedef enum bitcoinconsensus_error_t {
    bitcoinconsensus_ERR_OK = 0,
    bitcoinconsensus_ERR_TX_INDEX,
    bitcoinconsensus_ERR_TX_SIZE_MISMATCH,
    bitcoinconsensus_ERR_TX_DESERIALIZE,
    bitcoinconsensus_ERR_AMOUNT_REQUIRED,
    bitcoinconsensus_ERR_INVALID_FLAGS,
} bitcoinconsensus_error;

/* Script verification flags accepted by this interface (the libconsensus subset). */
enum {
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_NONE = 0,
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_P2SH = (1U << 0),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_DERSIG = (1U << 2),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_NULLDUMMY = (1U << 4),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKLOCKTIMEVERIFY = (1U << 9),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKSEQUENCEVERIFY = (1U << 10),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_WITNESS = (1U << 11),
    bitcoinconsensus_SCRIPT_FLAGS_VERIFY_ALL =
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_P2SH | bitcoinconsensus_SCRIPT_FLAGS_VERIFY_DERSIG |
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_NULLDUMMY |
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKLOCKTIMEVERIFY |
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_CHECKSEQUENCEVERIFY |
        bitcoinconsensus_SCRIPT_FLAGS_VERIFY_WITNESS,
};

int bitcoinconsensus_verify_script(const unsigned char* scriptPubKey, unsigned int scriptPubKeyLen,
                                   const unsigned char* txTo, unsigned int txToLen,
                                   unsigned int nIn, unsigned int flags, bitcoinconsensus_error* err);

int bitcoinconsensus_verify_script_with_amount(const unsigned char* scriptPubKey,
                                               unsigned int scriptPubKeyLen, int64_t amount,
                                               const unsigned char* txTo, unsigned int txToLen,
                                               unsigned int nIn, unsigned int flags,
                                               bitcoinconsensus_error* err);

unsigned int bitcoinconsensus_version(void);

/* One spend to verify.  Buffers are borrowed for the duration of the call only; items may share
 * the same txTo buffer (it is then deserialized once). */
typedef struct bcc_batch_item {
    const unsigned char* script_pubkey;
    unsigned int script_pubkey_len;
    int64_t amount;
    const unsigned char* tx_to;
    unsigned int tx_to_len;
    unsigned int n_in;
} bcc_batch_item;

/* Engine-specific error code, written ONLY by bitcoinconsensus_verify_batch under
 * BCC_DEVICE_FAILURE_ERROR, for items whose verdict the device could not deliver (never by the
 * single-item ABI, which aborts instead). */
#define BCC_ERR_DEVICE_FAILURE 6

/* Verifies n items with `flags`.  ret_out[i] / err_out[i] (err_out may be NULL) receive exactly
 * what bitcoinconsensus_verify_script_with_amount would return / write for item i.
 * Returns the number of valid items, or -1 if the device pipeline failed (BCC_DEVICE_FAILURE_ERROR
 * only; the default verifies such a round on the host): then
 * items the failed round left unfinished get ret_out 0 and err_out BCC_ERR_DEVICE_FAILURE, and
 * every other item carries its final result. */
long bitcoinconsensus_verify_batch(const bcc_batch_item* items, size_t n, unsigned int flags,
                                   int* ret_out, bitcoinconsensus_error* err_out);

#ifdef __cplusplus
}
#endif

#endif
