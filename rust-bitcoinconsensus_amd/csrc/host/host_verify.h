// Host-CPU evaluation of a device round (host_verify.cpp): the engine's own sighash jobs and lane
// verify code on the CPU, for device-failure fallback and small rounds.
#pragma once
#include <cstddef>
#include <cstdint>

#include "../pipeline.h"

namespace bcc {
namespace host {

// msg (32 bytes per row, entering as each row's initial message) receives every job's digest.
void host_sighash(const SighashJobs& jobs, uint8_t* msg);
// One tuple (tag 0 = rejected on the host; y ignored for 02/03): 1 valid.
int host_verify_tuple(uint8_t tag, const uint8_t* x32, const uint8_t* y32, const uint8_t* r32,
                      const uint8_t* s32, const uint8_t* m32);
void host_verify_rows(const TupleRows& rows, const uint8_t* msg, uint8_t* verdict, unsigned threads);
// gpu_verify_parts on the host: the same verdicts for the concatenation of P parts.
// The key-hash conditions of R (TupleRows::hrow / hprog, the device's key_hash_kernel): clears
// verdict[row] where HASH160(the row's key) != the program.
void apply_key_hashes(const TupleRows& R, uint8_t* verdict);
int host_verify_parts(const SighashJobs* const* jobs, const TupleRows* const* rows, size_t P,
                      uint8_t* verdict, unsigned threads);

size_t host_small_round();     // bcc_set_host_small_round (0: every round on the GPU)
bool host_fallback_enabled();  // bcc_set_device_failure_policy == BCC_DEVICE_FAILURE_HOST
void note_host_fallback();     // counts bcc_host_fallback_rounds

}  // namespace host
}  // namespace bcc
