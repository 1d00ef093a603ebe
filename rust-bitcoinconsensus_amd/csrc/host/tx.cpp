// Transaction deserializer (see tx.h).
#include "tx.h"

namespace bcc {
namespace host {

namespace {

constexpr uint64_t MAX_SIZE = 0x02000000;  // serialize.h:31

struct Reader {
    const uint8_t* p;
    size_t n, pos = 0;
    bool bad = false;
    const uint8_t* take(size_t k) {
        if (bad || k > n - pos) {
            bad = true;
            return nullptr;
        }
        const uint8_t* q = p + pos;
        pos += k;
        return q;
    }
    uint64_t le(int k) {
        const uint8_t* q = take((size_t)k);
        if (!q) return 0;
        uint64_t v = 0;
        for (int i = k - 1; i >= 0; i--) v = (v << 8) | q[i];
        return v;
    }
    // ReadCompactSize with range_check (serialize.h:318-347)
    uint64_t compact() {
        uint64_t c = le(1), v;
        if (bad) return 0;
        if (c < 253) {
            v = c;
        } else if (c == 253) {
            v = le(2);
            if (v < 253) bad = true;
        } else if (c == 254) {
            v = le(4);
            if (v < 0x10000u) bad = true;
        } else {
            v = le(8);
            if (v < 0x100000000ULL) bad = true;
        }
        if (v > MAX_SIZE) bad = true;
        return bad ? 0 : v;
    }
    Span bytes() {
        uint64_t k = compact();
        Span s;
        if (bad) return s;
        s.p = take((size_t)k);
        s.n = bad ? 0 : (size_t)k;
        return s;
    }
};

// The vin list after its compact-size count k has been read.
bool read_vin_items(Reader& r, std::vector<TxIn>& vin, uint64_t k) {
    if (r.bad || k > r.n - r.pos) return false;  // every element needs >= 1 byte: EOF anyway
    vin.resize((size_t)k);  // existing elements (and their witness capacity) are reused
    for (auto& in : vin) {
        in.witness.clear();
        in.prevout = r.take(36);
        in.script_sig = r.bytes();
        in.sequence = (uint32_t)r.le(4);
        if (r.bad) return false;
    }
    return true;
}

bool read_vin(Reader& r, std::vector<TxIn>& vin) { return read_vin_items(r, vin, r.compact()); }

bool read_vout(Reader& r, std::vector<TxOut>& vout) {
    uint64_t k = r.compact();
    if (r.bad || k > r.n - r.pos) return false;
    vout.resize((size_t)k);
    for (auto& o : vout) {
        size_t start = r.pos;
        o.value = (int64_t)r.le(8);
        o.script = r.bytes();
        if (r.bad) return false;
        o.ser.p = r.p + start;
        o.ser.n = r.pos - start;
    }
    return true;
}

}  // namespace

bool parse_tx(const uint8_t* data, size_t len, Tx& tx) {
    Reader r{data, len};
    // no clear(): vin / vout are resized in place, so a reused Tx keeps its elements and their
    // witness vectors' capacity (no per-input allocation when callers reuse Tx objects)
    tx.version = 0;
    tx.locktime = 0;
    tx.ser_size = 0;
    tx.version = (int32_t)(uint32_t)r.le(4);
    if (r.bad) return false;
    uint8_t flags = 0;
    const uint64_t k = r.compact();
    if (r.bad) return false;
    if (k == 0) {  // dummy (segwit marker) or an empty vin; vin is not shrunk before we know
        flags = (uint8_t)r.le(1);
        if (r.bad) return false;
        if (flags != 0) {
            if (!read_vin(r, tx.vin)) return false;
            if (!read_vout(r, tx.vout)) return false;
        } else {
            tx.vin.clear();
            tx.vout.clear();
        }
    } else {
        if (!read_vin_items(r, tx.vin, k)) return false;
        if (!read_vout(r, tx.vout)) return false;
    }
    if (flags & 1) {
        flags ^= 1;
        for (auto& in : tx.vin) {
            uint64_t k = r.compact();
            if (r.bad || k > r.n - r.pos) return false;
            in.witness.resize((size_t)k);
            for (auto& w : in.witness) {
                w = r.bytes();
                if (r.bad) return false;
            }
        }
        if (!tx.has_witness()) return false;  // "Superfluous witness record"
    }
    if (flags) return false;                  // "Unknown transaction optional data"
    tx.locktime = (uint32_t)r.le(4);
    if (r.bad) return false;
    tx.ser_size = r.pos;
    return true;
}

bool parse_txouts(const uint8_t* data, size_t len, std::vector<TxOut>& outs) {
    Reader r{data, len};
    outs.clear();
    return read_vout(r, outs) && r.pos == len;
}

void put_compact_size(std::vector<uint8_t>& out, uint64_t v) {
    if (v < 253) {
        out.push_back((uint8_t)v);
    } else if (v <= 0xFFFF) {
        out.push_back(253);
        for (int i = 0; i < 2; i++) out.push_back((uint8_t)(v >> (8 * i)));
    } else if (v <= 0xFFFFFFFFULL) {
        out.push_back(254);
        for (int i = 0; i < 4; i++) out.push_back((uint8_t)(v >> (8 * i)));
    } else {
        out.push_back(255);
        for (int i = 0; i < 8; i++) out.push_back((uint8_t)(v >> (8 * i)));
    }
}

}  // namespace host
}  // namespace bcc
