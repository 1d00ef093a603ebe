// Host side of hot-path stage (a): building SHA-256d *jobs* (preimage bytes) for the GPU.
// The host only serializes; every SHA-256 compression of a signature hash runs on the GPU
// (csrc/sighash.hip).
//
//   legacy preimage   CTransactionSignatureSerializer (interpreter.cpp:1273-1364) || hashtype
//                     incl. the SIGHASH_SINGLE bug -> uint256::ONE (interpreter.cpp:1627-1633)
//   BIP143 preimage   interpreter.cpp:1581-1625; hashPrevouts / hashSequence / hashOutputs are
//                     themselves SHA-256d of per-tx "aux" messages (interpreter.cpp:1366-1397,
//                     PrecomputedTransactionData::Init :1422-1472) whose digests the GPU patches
//                     into the preimage before hashing it.
// Also: the CPubKey length filter, lax-DER parsing and signature normalisation that precede
// secp256k1_ecdsa_verify in CPubKey::Verify (pubkey.cpp:28-168, 191-207).
#pragma once
#include <cstdint>
#include <vector>

#include "script.h"
#include "tx.h"

namespace bcc {
namespace host {

// Aux message kinds per tx (BIP143 precompute)
enum AuxKind { AUX_PREVOUTS = 0, AUX_SEQUENCES = 1, AUX_OUTPUTS = 2 };

void build_aux_message(const Tx& tx, AuxKind kind, std::vector<uint8_t>& out);

// Legacy preimage (serializer || nHashType as int32 LE).  Returns false for the SINGLE bug
// (the sighash is then the constant ONE and no hashing happens).
bool build_legacy_preimage(const Tx& tx, unsigned nin, const Bytes& script_code, int hashtype,
                           std::vector<uint8_t>& out);

// The device-assembled form of a legacy SIGHASH_ALL preimage (pipeline.h TplJob):
// legacy_template = the tx serialized with every scriptSig empty (no witness, no hashtype);
// legacy_template_pos = offset of input nin's empty-script length byte in it;
// script_code_field = compactsize || scriptCode without OP_CODESEPARATORs (SerializeScriptCode).
// legacy_all_type: hashtypes whose preimage has that form (not NONE / SINGLE / ANYONECANPAY).
void build_legacy_template(const Tx& tx, std::vector<uint8_t>& out);
size_t legacy_template_pos(const Tx& tx, unsigned nin);
size_t legacy_template_len(const Tx& tx);  // build_legacy_template's output size
void build_script_code_field(const Bytes& script_code, std::vector<uint8_t>& out);
inline bool legacy_all_type(int hashtype) {
    return (hashtype & 0x80) == 0 && (hashtype & 0x1f) != 2 && (hashtype & 0x1f) != 3;
}

// BIP143 preimage with zeroed 32-byte slots for hashPrevouts (offset 4), hashSequence (offset 36)
// and hashOutputs (offset len-40).  need[k] says whether slot k must be patched with aux digest k
// (AuxKind order; for SIGHASH_SINGLE with nin < vout.size() slot 2 takes the digest of the
// single output, which the caller adds as an extra aux message: *single_output).
struct Bip143Job {
    std::vector<uint8_t> preimage;
    bool need[3];
    size_t off[3];
    bool single_output;  // slot 2 = SHA256d(vout[nin]) instead of hashOutputs
};
void build_bip143_preimage(const Tx& tx, unsigned nin, const Bytes& script_code, int hashtype,
                           int64_t amount, Bip143Job& job);

// CPubKey(vch).IsValid(): header 02/03 with 33 bytes, 04/06/07 with 65 bytes (pubkey.h:58-94)
bool pubkey_size_valid(const uint8_t* p, size_t n);

// ecdsa_signature_parse_der_lax (pubkey.cpp:28-168) + parse_compact overflow rule: returns false
// on malformed input; on success r/s (big-endian) are zero if either integer overflowed / >= n.
bool der_parse_lax(const uint8_t* sig, size_t len, uint8_t r[32], uint8_t s[32]);

}  // namespace host
}  // namespace bcc
