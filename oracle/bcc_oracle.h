/* oracle/bcc_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C restatement of the reference's signature hot path (SURVEY.md §8a rows a3-a6, a9-a18,
 * a20). It is the CHECKER for the HIP kernels: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product (rust-bitcoinconsensus_amd/) never links it.
 *
 * Parity of this restatement is pinned against the reference itself (oracle/_ref, compiled from
 * /root/reference by oracle/Makefile) and the reference's own fixtures (tests/golden/).
 *
 * Conventions: every 32-byte value is big-endian bytes (the reference's b32 convention), except
 * sighash outputs which are the raw SHA-256d bytes (uint256::begin()).
 */
#ifndef BCC_ORACLE_H
#define BCC_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* SHA-256 / SHA-256d (crypto/sha256.cpp:637-679, hash.h:100-137) */
void bcco_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
void bcco_sha256d(const uint8_t* msg, size_t len, uint8_t out[32]);

/* Lax DER (pubkey.cpp:28-168). Returns 0 on a malformed encoding; returns 1 otherwise, with
 * r = s = 0 when either integer overflows 32 bytes or is >= n. */
int bcco_der_parse_lax(const uint8_t* sig, size_t len, uint8_t r[32], uint8_t s[32]);

/* secp256k1_ec_pubkey_parse (secp256k1.c:277-293, eckey_impl.h:17-35) incl. the CPubKey
 * length/header filter (pubkey.h:58-94). Returns 1 and the affine point on success. */
int bcco_pubkey_parse(const uint8_t* pub, size_t len, uint8_t x[32], uint8_t y[32]);

/* secp256k1_ecdsa_sig_verify (ecdsa_impl.h:207-275) on an affine key and raw (r, s, msg32).
 * Includes the r,s != 0 test, m = msg mod n, and the xr / xr+n acceptance rule. s is NOT
 * normalized here (verdict is invariant under s -> n-s). */
int bcco_ecdsa_verify_raw(const uint8_t qx[32], const uint8_t qy[32], const uint8_t r[32],
                          const uint8_t s[32], const uint8_t msg32[32]);

/* CPubKey::Verify (pubkey.cpp:191-207): pub bytes, raw sighash, DER sig WITHOUT hashtype. */
int bcco_pubkey_verify(const uint8_t* pub, size_t publen, const uint8_t hash32[32],
                       const uint8_t* sig, size_t siglen);

/* secp256k1_schnorrsig_verify (modules/schnorrsig/main_impl.h:190-237) with xonly parse
 * (modules/extrakeys/main_impl.h:21-39). */
int bcco_schnorr_verify(const uint8_t sig64[64], const uint8_t msg32[32], const uint8_t xonly32[32]);

/* k*G, affine output (for generator/fixture checks). Returns 0 if k == 0 mod n. */
int bcco_ecmult_gen(const uint8_t k32[32], uint8_t x[32], uint8_t y[32]);

/* Signature hash (interpreter.cpp:1576-1642) over a serialized tx.
 * sigversion 0 = BASE (legacy, CTransactionSignatureSerializer :1273-1364 incl. the SINGLE bug),
 * 1 = WITNESS_V0 (BIP143). scriptCode is given as-is (after FindAndDelete / codeseparator
 * positioning by the interpreter); legacy serialization strips OP_CODESEPARATOR opcodes.
 * Returns 1 on success, 0 if the tx does not parse or nIn is out of range. */
int bcco_sighash(const uint8_t* tx, size_t txlen, unsigned nIn, const uint8_t* script,
                 size_t scriptlen, int hashtype, int64_t amount, int sigversion, uint8_t out32[32]);

/* BIP341 / BIP342 SignatureHashSchnorr (interpreter.cpp:1491-1574) over a serialized tx and its
 * spent outputs (a serialized std::vector<CTxOut>, one per input: PrecomputedTransactionData::Init
 * :1422-1472).  sigversion 0 = TAPROOT (key path), 1 = TAPSCRIPT (tapleaf32 + codesep_pos used).
 * annex = the annex witness element incl. its 0x50 byte, or NULL when absent.  Returns 1 with the
 * hash, 0 where the reference returns false (bad hash_type, SINGLE without a matching output),
 * -1 if the tx (all tx_len bytes, the bitcoinconsensus.cpp:91-92 size rule) or the spent outputs
 * do not parse, their counts differ, nIn is out of range or the tx data would not be BIP341-ready
 * (no witness-bearing input spends a 34-byte OP_1 script, interpreter.cpp:1436-1452). */
int bcco_sighash_schnorr(const uint8_t* tx, size_t txlen, const uint8_t* spent, size_t spentlen,
                         unsigned nIn, int hash_type, int sigversion, const uint8_t* annex,
                         size_t annexlen, const uint8_t tapleaf32[32], uint32_t codesep_pos,
                         uint8_t out32[32]);

/* GenericTransactionSignatureChecker::CheckSchnorrSignature (interpreter.cpp:1678-1704): 1 valid;
 * 0 invalid with *serror = 44 SCHNORR_SIG_SIZE / 45 SCHNORR_SIG_HASHTYPE / 46 SCHNORR_SIG
 * (script_error.h:73-75); -1 for inputs bcco_sighash_schnorr refuses. */
int bcco_taproot_check(const uint8_t* tx, size_t txlen, const uint8_t* spent, size_t spentlen,
                       unsigned nIn, const uint8_t* sig, size_t siglen, const uint8_t pk32[32],
                       int sigversion, const uint8_t* annex, size_t annexlen,
                       const uint8_t tapleaf32[32], uint32_t codesep_pos, int* serror,
                       uint8_t* sighash32);

#ifdef __cplusplus
}
#endif
#endif
