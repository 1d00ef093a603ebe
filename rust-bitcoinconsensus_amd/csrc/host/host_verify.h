// Host-CPU evaluation of a device round (host_verify.cpp): the engine's own sighash jobs and lane
// verify code on the CPU, for device-failure fallback and small rounds.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../pipeline.h"

namespace bcc {
namespace host {

// msg (32 bytes per row, entering as each row's initial message) receives every job's digest.
void host_sighash(const SighashJobs& jobs, uint8_t* msg);
// The sighash of legacy template job t over its template / code blobs (K3' on the host): from the
// midstate at its splice block when t carries TPL_MID (pipeline.h), else from the IV.
void tpl_job_sighash(const uint8_t* tpl, const uint8_t* code, const TplJob& t, uint8_t out[32]);
// mid = the tpl_mid_count(len) SHA-256 midstates of template T (8 native-order words each).
void tpl_midstates(const uint8_t* T, uint32_t len, std::vector<uint32_t>& mid);
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
