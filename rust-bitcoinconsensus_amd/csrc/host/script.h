// Host-kept script interpreter (SURVEY §2b "Script interpreter", north star: "keeps the
// interpreter on the CPU").  Restates the consensus behaviour of
//   EvalScript            script/interpreter.cpp:431-1259
//   VerifyScript          script/interpreter.cpp:1937-2056
//   VerifyWitnessProgram  script/interpreter.cpp:1855-1935 (witness v0; v1+ pass unchecked
//                         because SCRIPT_VERIFY_TAPROOT is not a libconsensus flag)
//   ExecuteWitnessScript  script/interpreter.cpp:1794-1832
//   CScriptNum            script/script.h:218-391
// for the libconsensus flag set (bitcoinconsensus.h:178-190: P2SH, DERSIG, NULLDUMMY, CLTV,
// CSV, WITNESS).  Every ECDSA check goes through SigChecker::check_ecdsa — the deferral seam
// (BaseSignatureChecker::CheckECDSASignature, interpreter.h:227) where the batch engine records
// tuples for the GPU instead of verifying them.
#pragma once
#include <cstdint>
#include <vector>

#include "pool.h"
#include "tx.h"

namespace bcc {
namespace host {

// interpreter byte vectors (stack elements, script codes) on the small-block pool (pool.h)
typedef std::vector<uint8_t, PoolAlloc<uint8_t>> Bytes;

enum SigVersion { SIGVERSION_BASE = 0, SIGVERSION_WITNESS_V0 = 1 };

// libconsensus flag bits (script/interpreter.h:45-141)
enum : unsigned {
    FLAG_P2SH = 1u << 0,
    FLAG_DERSIG = 1u << 2,
    FLAG_NULLDUMMY = 1u << 4,
    FLAG_CHECKLOCKTIMEVERIFY = 1u << 9,
    FLAG_CHECKSEQUENCEVERIFY = 1u << 10,
    FLAG_WITNESS = 1u << 11,
    FLAGS_VERIFY_ALL = FLAG_P2SH | FLAG_DERSIG | FLAG_NULLDUMMY | FLAG_CHECKLOCKTIMEVERIFY |
                       FLAG_CHECKSEQUENCEVERIFY | FLAG_WITNESS,
};

// A subset of ScriptError (script/script_error.h) sufficient to report why a script failed.
enum ScriptErr {
    SERR_OK = 0,
    SERR_UNKNOWN,
    SERR_EVAL_FALSE,
    SERR_OP_RETURN,
    SERR_SCRIPT_SIZE,
    SERR_PUSH_SIZE,
    SERR_OP_COUNT,
    SERR_STACK_SIZE,
    SERR_SIG_COUNT,
    SERR_PUBKEY_COUNT,
    SERR_VERIFY,
    SERR_EQUALVERIFY,
    SERR_CHECKMULTISIGVERIFY,
    SERR_CHECKSIGVERIFY,
    SERR_NUMEQUALVERIFY,
    SERR_BAD_OPCODE,
    SERR_DISABLED_OPCODE,
    SERR_INVALID_STACK_OPERATION,
    SERR_INVALID_ALTSTACK_OPERATION,
    SERR_UNBALANCED_CONDITIONAL,
    SERR_NEGATIVE_LOCKTIME,
    SERR_UNSATISFIED_LOCKTIME,
    SERR_SIG_DER,
    SERR_SIG_PUSHONLY,
    SERR_SIG_NULLDUMMY,
    SERR_CLEANSTACK,
    SERR_WITNESS_PROGRAM_WRONG_LENGTH,
    SERR_WITNESS_PROGRAM_WITNESS_EMPTY,
    SERR_WITNESS_PROGRAM_MISMATCH,
    SERR_WITNESS_MALLEATED,
    SERR_WITNESS_MALLEATED_P2SH,
    SERR_WITNESS_UNEXPECTED,
};

// The deferral seam.  check_ecdsa receives exactly what BaseSignatureChecker::CheckECDSASignature
// receives: the full signature push (DER || hashtype), the pubkey push, the scriptCode (after
// FindAndDelete for BASE) and the sigversion.
class SigChecker {
public:
    virtual ~SigChecker() {}
    virtual bool check_ecdsa(const Bytes& sig, const Bytes& pub, const Bytes& script_code,
                             SigVersion sv) = 0;
    // A check the script may consult later in the same CHECKMULTISIG (a candidate (sig, key)
    // pair); a batching checker may queue it now.  Must not change any verdict.
    virtual void hint_ecdsa(const Bytes&, const Bytes&, const Bytes&, SigVersion) {}
    // Offer EVERY candidate pair of a CHECKMULTISIG, not only when there are few: a batching
    // checker turns this on for items that already needed a re-run, so that the key advance of
    // an m-of-n with many keys costs at most one more device round.
    virtual bool hint_all() const { return false; }
    // HASH160 of `p` if the checker already holds it (computed ahead in a batch for exactly these
    // bytes), else nullptr; OP_HASH160 then uses it instead of hashing again.
    virtual const uint8_t* cached_hash160(const uint8_t*, size_t) const { return nullptr; }
    // The <20> OP_EQUALVERIFY of a key-hash spend (P2WPKH, P2PKH): HASH160(key) == prog20.  A
    // batching checker may take it over: it returns true and the script goes on as if the hashes
    // matched; the checker then ties the condition to the NEXT check_ecdsa of this run (the
    // check's verdict becomes "signature valid AND hashes match").  key_hash_taken() after that
    // check_ecdsa says whether it did; when not, the script compares the hash itself before using
    // the check's result.  false (the default): the script hashes now.
    virtual bool defer_key_hash(const uint8_t*, size_t, const uint8_t*) { return false; }
    virtual bool key_hash_taken() { return false; }
    virtual bool check_locktime(int64_t n) = 0;
    virtual bool check_sequence(int64_t n) = 0;
};

// Lock-time rules of GenericTransactionSignatureChecker (interpreter.cpp:1706-1788).
bool tx_check_locktime(const Tx& tx, unsigned nin, int64_t n);
bool tx_check_sequence(const Tx& tx, unsigned nin, int64_t n);

bool verify_script(const Span& script_sig, const Span& spk, const std::vector<Span>& witness,
                   unsigned flags, SigChecker& checker, ScriptErr* err);

// helpers shared with the sighash / batch code
bool script_get_op(const uint8_t* s, size_t n, size_t& pc, uint8_t& op, const uint8_t** data,
                   size_t* datalen);
bool is_valid_signature_encoding(const Bytes& sig);   // interpreter.cpp:107-170 (BIP66)

}  // namespace host
}  // namespace bcc
