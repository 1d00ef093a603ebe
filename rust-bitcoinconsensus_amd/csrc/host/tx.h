// Transaction model + wire-format deserializer (host-kept, SURVEY §2b "Tx model").
// Restates UnserializeTransaction (primitives/transaction.h:188-224) and the CompactSize /
// vector rules of serialize.h:318-347 (canonical sizes, MAX_SIZE = 0x02000000).
// The parsed form keeps pointers into the caller's buffer: no copies of scripts or witnesses.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace bcc {
namespace host {

struct Span {
    const uint8_t* p = nullptr;
    size_t n = 0;
    const uint8_t* begin() const { return p; }
    const uint8_t* end() const { return p + n; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
};

struct TxIn {
    const uint8_t* prevout;  // 36 bytes: txid (32) || vout (4, LE)
    Span script_sig;
    uint32_t sequence;
    std::vector<Span> witness;
};

struct TxOut {
    int64_t value;
    Span script;
    Span ser;  // the serialized CTxOut bytes (value || compactsize || script)
};

struct Tx {
    int32_t version = 0;
    std::vector<TxIn> vin;
    std::vector<TxOut> vout;
    uint32_t locktime = 0;
    size_t ser_size = 0;  // bytes consumed == GetSerializeSize(tx, PROTOCOL_VERSION)
    bool has_witness() const {
        for (const auto& i : vin)
            if (!i.witness.empty()) return true;
        return false;
    }
};

// Returns false where the reference's deserializer throws (std::ios_base::failure).
bool parse_tx(const uint8_t* data, size_t len, Tx& tx);

// A serialized std::vector<CTxOut> occupying exactly len bytes (the spent outputs handed to
// PrecomputedTransactionData::Init, interpreter.cpp:1422-1472).  False where it would not parse.
bool parse_txouts(const uint8_t* data, size_t len, std::vector<TxOut>& outs);

// CompactSize writer (serialize.h WriteCompactSize)
void put_compact_size(std::vector<uint8_t>& out, uint64_t v);

}  // namespace host
}  // namespace bcc
