// Sighash preimage builders + signature/pubkey front-end filters (see sighash.h).
#include "sighash.h"

#include <cstring>

namespace bcc {
namespace host {

namespace {

void put_le(std::vector<uint8_t>& o, uint64_t v, int k) {
    for (int i = 0; i < k; i++) o.push_back((uint8_t)(v >> (8 * i)));
}
void put(std::vector<uint8_t>& o, const uint8_t* p, size_t n) { o.insert(o.end(), p, p + n); }

// SerializeScriptCode (interpreter.cpp:1293-1312): drop OP_CODESEPARATORs; note the length
// prefix counts separators over the parseable prefix while the bytes stop where parsing stopped.
void put_script_code(std::vector<uint8_t>& o, const Bytes& sc) {
    size_t pc = 0, ncs = 0;
    uint8_t op;
    while (script_get_op(sc.data(), sc.size(), pc, op, nullptr, nullptr))
        if (op == 0xab) ncs++;
    put_compact_size(o, sc.size() - ncs);
    size_t begin = 0;
    pc = 0;
    while (script_get_op(sc.data(), sc.size(), pc, op, nullptr, nullptr)) {
        if (op == 0xab) {
            put(o, sc.data() + begin, pc - begin - 1);
            begin = pc;
        }
    }
    if (begin != sc.size()) put(o, sc.data() + begin, pc - begin);
}

const uint8_t N_BE[32] = {0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF, 0xFF,
                          0xFF, 0xFF, 0xFF, 0xFF, 0xFE, 0xBA, 0xAE, 0xDC, 0xE6, 0xAF, 0x48,
                          0xA0, 0x3B, 0xBF, 0xD2, 0x5E, 0x8C, 0xD0, 0x36, 0x41, 0x41};

bool ge_n(const uint8_t* v) { return memcmp(v, N_BE, 32) >= 0; }

// integer length field of the lax parser
bool der_len(const uint8_t* in, size_t inlen, size_t& pos, size_t& out) {
    if (pos == inlen) return false;
    size_t lenbyte = in[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (lenbyte > inlen - pos) return false;
        while (lenbyte > 0 && in[pos] == 0) {
            pos++;
            lenbyte--;
        }
        if (lenbyte >= 4) return false;
        size_t v = 0;
        while (lenbyte > 0) {
            v = (v << 8) + in[pos];
            pos++;
            lenbyte--;
        }
        out = v;
    } else {
        out = lenbyte;
    }
    return true;
}

}  // namespace

void build_aux_message(const Tx& tx, AuxKind kind, std::vector<uint8_t>& out) {
    out.clear();
    if (kind == AUX_PREVOUTS) {
        for (const auto& in : tx.vin) put(out, in.prevout, 36);
    } else if (kind == AUX_SEQUENCES) {
        for (const auto& in : tx.vin) put_le(out, in.sequence, 4);
    } else {
        for (const auto& o : tx.vout) put(out, o.ser.p, o.ser.n);
    }
}

bool build_legacy_preimage(const Tx& tx, unsigned nin, const Bytes& sc, int hashtype,
                           std::vector<uint8_t>& o) {
    const bool acp = (hashtype & 0x80) != 0;
    const bool single = (hashtype & 0x1f) == 3, none = (hashtype & 0x1f) == 2;
    if (single && nin >= tx.vout.size()) return false;  // SIGHASH_SINGLE bug -> ONE
    o.clear();
    put_le(o, (uint32_t)tx.version, 4);
    size_t nins = acp ? 1 : tx.vin.size();
    put_compact_size(o, nins);
    for (size_t k = 0; k < nins; k++) {
        size_t i = acp ? nin : k;
        put(o, tx.vin[i].prevout, 36);
        if (i != nin) put_compact_size(o, 0);
        else put_script_code(o, sc);
        if (i != nin && (single || none)) put_le(o, 0, 4);
        else put_le(o, tx.vin[i].sequence, 4);
    }
    size_t nouts = none ? 0 : (single ? nin + 1 : tx.vout.size());
    put_compact_size(o, nouts);
    for (size_t k = 0; k < nouts; k++) {
        if (single && k != nin) {  // CTxOut(): nValue = -1, empty script
            put_le(o, (uint64_t)(int64_t)-1, 8);
            put_compact_size(o, 0);
        } else {
            put(o, tx.vout[k].ser.p, tx.vout[k].ser.n);
        }
    }
    put_le(o, tx.locktime, 4);
    put_le(o, (uint32_t)hashtype, 4);
    return true;
}

void build_legacy_template(const Tx& tx, std::vector<uint8_t>& o) {
    o.clear();
    put_le(o, (uint32_t)tx.version, 4);
    put_compact_size(o, tx.vin.size());
    for (const auto& in : tx.vin) {
        put(o, in.prevout, 36);
        o.push_back(0);
        put_le(o, in.sequence, 4);
    }
    put_compact_size(o, tx.vout.size());
    for (const auto& out : tx.vout) put(o, out.ser.p, out.ser.n);
    put_le(o, tx.locktime, 4);
}

static size_t compact_size_len(size_t n) { return n < 0xfd ? 1 : n <= 0xffff ? 3 : n <= 0xffffffffu ? 5 : 9; }

size_t legacy_template_len(const Tx& tx) {
    size_t out = 0;
    for (const auto& o : tx.vout) out += o.ser.n;
    return 4 + compact_size_len(tx.vin.size()) + 41 * tx.vin.size() +
           compact_size_len(tx.vout.size()) + out + 4;
}

size_t legacy_template_pos(const Tx& tx, unsigned nin) {
    const size_t n = tx.vin.size();
    const size_t cs = n < 0xfd ? 1 : n <= 0xffff ? 3 : n <= 0xffffffffu ? 5 : 9;
    return 4 + cs + 41 * (size_t)nin + 36;
}

void build_script_code_field(const Bytes& sc, std::vector<uint8_t>& o) {
    o.clear();
    put_script_code(o, sc);
}

void build_bip143_preimage(const Tx& tx, unsigned nin, const Bytes& sc, int hashtype,
                           int64_t amount, Bip143Job& job) {
    const bool acp = (hashtype & 0x80) != 0;
    const int base = hashtype & 0x1f;
    const bool single = base == 3, none = base == 2;
    job.need[AUX_PREVOUTS] = !acp;
    job.need[AUX_SEQUENCES] = !acp && !single && !none;
    job.single_output = single && nin < tx.vout.size();
    job.need[AUX_OUTPUTS] = (!single && !none) || job.single_output;
    auto& o = job.preimage;
    o.clear();
    o.reserve(160 + sc.size());
    put_le(o, (uint32_t)tx.version, 4);
    job.off[AUX_PREVOUTS] = o.size();
    o.insert(o.end(), 32, 0);
    job.off[AUX_SEQUENCES] = o.size();
    o.insert(o.end(), 32, 0);
    put(o, tx.vin[nin].prevout, 36);
    put_compact_size(o, sc.size());
    put(o, sc.data(), sc.size());
    put_le(o, (uint64_t)amount, 8);
    put_le(o, tx.vin[nin].sequence, 4);
    job.off[AUX_OUTPUTS] = o.size();
    o.insert(o.end(), 32, 0);
    put_le(o, tx.locktime, 4);
    put_le(o, (uint32_t)hashtype, 4);
}

bool pubkey_size_valid(const uint8_t* p, size_t n) {
    if (n == 0) return false;
    if (p[0] == 2 || p[0] == 3) return n == 33;
    if (p[0] == 4 || p[0] == 6 || p[0] == 7) return n == 65;
    return false;
}

bool der_parse_lax(const uint8_t* in, size_t inlen, uint8_t r[32], uint8_t s[32]) {
    size_t pos = 0, rpos, rlen, spos, slen, lenbyte;
    uint8_t tmp[64];
    memset(tmp, 0, 64);
    memset(r, 0, 32);
    memset(s, 0, 32);
    if (pos == inlen || in[pos] != 0x30) return false;
    pos++;
    if (pos == inlen) return false;
    lenbyte = in[pos++];
    if (lenbyte & 0x80) {
        lenbyte -= 0x80;
        if (lenbyte > inlen - pos) return false;
        pos += lenbyte;
    }
    if (pos == inlen || in[pos] != 0x02) return false;
    pos++;
    if (!der_len(in, inlen, pos, rlen)) return false;
    if (rlen > inlen - pos) return false;
    rpos = pos;
    pos += rlen;
    if (pos == inlen || in[pos] != 0x02) return false;
    pos++;
    if (!der_len(in, inlen, pos, slen)) return false;
    if (slen > inlen - pos) return false;
    spos = pos;
    bool overflow = false;
    while (rlen > 0 && in[rpos] == 0) {
        rlen--;
        rpos++;
    }
    if (rlen > 32) overflow = true;
    else memcpy(tmp + 32 - rlen, in + rpos, rlen);
    while (slen > 0 && in[spos] == 0) {
        slen--;
        spos++;
    }
    if (slen > 32) overflow = true;
    else memcpy(tmp + 64 - slen, in + spos, slen);
    if (!overflow && (ge_n(tmp) || ge_n(tmp + 32))) overflow = true;  // parse_compact
    if (overflow) memset(tmp, 0, 64);
    memcpy(r, tmp, 32);
    memcpy(s, tmp + 32, 32);
    return true;
}

}  // namespace host
}  // namespace bcc
