// Internal interface of the batch engine (engine.cpp), shared with the workload builder.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../pipeline.h"
#include "bitcoinconsensus.h"

namespace bcc {
namespace host {

// Deserializes and checks the items (flags / deserialize / index / size, in reference order) and
// runs the interpreter once with the deferring checker.  jobs / rows receive every deferred ECDSA
// check (the first GPU round of bitcoinconsensus_verify_batch); tuple_item[k] = item of row k.
// Returns the number of deferred tuples.
size_t build_first_round(const bcc_batch_item* items, size_t n, unsigned flags, SighashJobs& jobs,
                         TupleRows& rows, std::vector<uint32_t>* tuple_item = nullptr);

// One signature check's sighash inputs (tests / debugging of the sighash kernels): the spending
// tx, the input index, the scriptCode as GenericTransactionSignatureChecker receives it, the full
// 32-bit hash type, the spent amount (BIP143) and the SigVersion (0 BASE, 1 WITNESS_V0).
struct SighashCheck {
    const uint8_t* tx;
    size_t tx_len;
    const uint8_t* code;
    size_t code_len;
    unsigned nin;
    int hashtype;
    int64_t amount;
    int sigversion;
};

// Builds the device sighash jobs of n checks exactly as the deferring checker builds them for a
// deferred tuple (one row per check, msg = ONE unless a kernel overwrites it).  Returns n, or the
// index of the first check whose tx does not parse / whose nin or sigversion is out of range.
size_t build_sighash_checks(const SighashCheck* checks, size_t n, SighashJobs& jobs,
                            TupleRows& rows);

// Appends src (jobs + rows) to dst, fixing offsets / indices.
void append_round(SighashJobs& dst, TupleRows& dst_rows, const SighashJobs& src,
                  const TupleRows& src_rows);

// A pending bcc_debug_fail_device_rounds fault, consumed (its HIP error code), else 0: the staged
// rounds (tuples.cpp) take it as a failed staging, as device_round does for a failed round.
int injected_device_fault();

// One device round of P parts on `dev` with the engine's failure handling: one retry on a fresh
// device batch for a transient HIP error (*retries), then the device failure policy: the parts are
// verified on the host CPU (*host_rounds, bcc_host_fallback_rounds) or the error is returned.
// `who` names the entry point in the stderr log.  `late` (optional): rows whose message the host
// delivers during the round (pipeline.h LateMsgFill); it is also called before a host fallback, so
// those rows' host messages are complete before the host verifies them.
int resilient_round(int dev, const SighashJobs* const* pj, const TupleRows* const* pr, size_t P,
                    uint8_t* verdict, double* stage_s, size_t* retries, size_t* host_rounds,
                    const char* who, const LateMsgFill* late = nullptr);

// Frees the calling thread's Taproot job buffers (host/taproot.cpp).
void taproot_release_thread_state();

// The SigMsg digests of a part's device-built Taproot jobs computed on the host (the CPU twin of
// sighash.hip taproot_tx_kernel + taproot_msg_kernel: tests, stub device): msg + 32 row.
void taproot_dev_sigmsg_host(const TaprootTxJobs& jobs, uint8_t* msg);

}  // namespace host
}  // namespace bcc
