// Host script interpreter (see script.h for the reference line map).
#include "script.h"

#include <cstring>
#include <stdexcept>

#include "hashes.h"

namespace bcc {
namespace host {

namespace {

enum Op : uint8_t {
    OP_0 = 0x00, OP_PUSHDATA1 = 0x4c, OP_PUSHDATA2 = 0x4d, OP_PUSHDATA4 = 0x4e, OP_1NEGATE = 0x4f,
    OP_1 = 0x51, OP_16 = 0x60, OP_NOP = 0x61, OP_IF = 0x63, OP_NOTIF = 0x64, OP_ELSE = 0x67,
    OP_ENDIF = 0x68, OP_VERIFY = 0x69, OP_RETURN = 0x6a, OP_TOALTSTACK = 0x6b,
    OP_FROMALTSTACK = 0x6c, OP_2DROP = 0x6d, OP_2DUP = 0x6e, OP_3DUP = 0x6f, OP_2OVER = 0x70,
    OP_2ROT = 0x71, OP_2SWAP = 0x72, OP_IFDUP = 0x73, OP_DEPTH = 0x74, OP_DROP = 0x75,
    OP_DUP = 0x76, OP_NIP = 0x77, OP_OVER = 0x78, OP_PICK = 0x79, OP_ROLL = 0x7a, OP_ROT = 0x7b,
    OP_SWAP = 0x7c, OP_TUCK = 0x7d, OP_CAT = 0x7e, OP_SUBSTR = 0x7f, OP_LEFT = 0x80,
    OP_RIGHT = 0x81, OP_SIZE = 0x82, OP_INVERT = 0x83, OP_AND = 0x84, OP_OR = 0x85, OP_XOR = 0x86,
    OP_EQUAL = 0x87, OP_EQUALVERIFY = 0x88, OP_1ADD = 0x8b, OP_1SUB = 0x8c, OP_2MUL = 0x8d,
    OP_2DIV = 0x8e, OP_NEGATE = 0x8f, OP_ABS = 0x90, OP_NOT = 0x91, OP_0NOTEQUAL = 0x92,
    OP_ADD = 0x93, OP_SUB = 0x94, OP_MUL = 0x95, OP_DIV = 0x96, OP_MOD = 0x97, OP_LSHIFT = 0x98,
    OP_RSHIFT = 0x99, OP_BOOLAND = 0x9a, OP_BOOLOR = 0x9b, OP_NUMEQUAL = 0x9c,
    OP_NUMEQUALVERIFY = 0x9d, OP_NUMNOTEQUAL = 0x9e, OP_LESSTHAN = 0x9f, OP_GREATERTHAN = 0xa0,
    OP_LESSTHANOREQUAL = 0xa1, OP_GREATERTHANOREQUAL = 0xa2, OP_MIN = 0xa3, OP_MAX = 0xa4,
    OP_WITHIN = 0xa5, OP_RIPEMD160 = 0xa6, OP_SHA1 = 0xa7, OP_SHA256 = 0xa8, OP_HASH160 = 0xa9,
    OP_HASH256 = 0xaa, OP_CODESEPARATOR = 0xab, OP_CHECKSIG = 0xac, OP_CHECKSIGVERIFY = 0xad,
    OP_CHECKMULTISIG = 0xae, OP_CHECKMULTISIGVERIFY = 0xaf, OP_NOP1 = 0xb0,
    OP_CHECKLOCKTIMEVERIFY = 0xb1, OP_CHECKSEQUENCEVERIFY = 0xb2, OP_NOP4 = 0xb3, OP_NOP10 = 0xb9,
};

constexpr size_t MAX_SCRIPT_ELEMENT_SIZE = 520;
constexpr int MAX_OPS_PER_SCRIPT = 201;
constexpr int MAX_PUBKEYS_PER_MULTISIG = 20;
constexpr size_t MAX_SCRIPT_SIZE = 10000;
constexpr size_t MAX_STACK_SIZE = 1000;
constexpr int64_t LOCKTIME_THRESHOLD = 500000000;
constexpr uint32_t SEQUENCE_FINAL = 0xffffffffu;
constexpr uint32_t SEQUENCE_LOCKTIME_DISABLE_FLAG = 1u << 31;
constexpr uint32_t SEQUENCE_LOCKTIME_TYPE_FLAG = 1u << 22;
constexpr uint32_t SEQUENCE_LOCKTIME_MASK = 0x0000ffffu;

struct ScriptNumError : std::runtime_error {
    ScriptNumError() : std::runtime_error("scriptnum") {}
};

// CScriptNum semantics (script.h:218-391), fRequireMinimal is never set by libconsensus flags.
int64_t num_decode(const Bytes& v, size_t max_size = 4) {
    if (v.size() > max_size) throw ScriptNumError();
    if (v.empty()) return 0;
    int64_t r = 0;
    for (size_t i = 0; i < v.size(); i++) r |= (int64_t)v[i] << (8 * i);
    if (v.back() & 0x80) return -((int64_t)(r & ~(int64_t)(0x80ULL << (8 * (v.size() - 1)))));
    return r;
}

Bytes num_encode(int64_t value) {
    Bytes out;
    if (value == 0) return out;
    bool neg = value < 0;
    uint64_t a = neg ? ~(uint64_t)value + 1 : (uint64_t)value;
    while (a) {
        out.push_back((uint8_t)(a & 0xff));
        a >>= 8;
    }
    if (out.back() & 0x80) out.push_back(neg ? 0x80 : 0);
    else if (neg) out.back() |= 0x80;
    return out;
}

int num_getint(int64_t v) {
    if (v > 2147483647LL) return 2147483647;
    if (v < -2147483648LL) return (int)-2147483648LL;
    return (int)v;
}

bool cast_to_bool(const uint8_t* v, size_t n) {
    for (size_t i = 0; i < n; i++) {
        if (v[i] != 0) {
            if (i == n - 1 && v[i] == 0x80) return false;  // negative zero
            return true;
        }
    }
    return false;
}

bool cast_to_bool(const Bytes& v) { return cast_to_bool(v.data(), v.size()); }

bool fail(ScriptErr* e, ScriptErr code) {
    if (e) *e = code;
    return false;
}

// CScript() << data : minimal push-opcode encoding (script.h:457-484)
void push_data(Bytes& s, const uint8_t* d, size_t n) {
    if (n < OP_PUSHDATA1) {
        s.push_back((uint8_t)n);
    } else if (n <= 0xff) {
        s.push_back(OP_PUSHDATA1);
        s.push_back((uint8_t)n);
    } else if (n <= 0xffff) {
        s.push_back(OP_PUSHDATA2);
        s.push_back((uint8_t)n);
        s.push_back((uint8_t)(n >> 8));
    } else {
        s.push_back(OP_PUSHDATA4);
        for (int i = 0; i < 4; i++) s.push_back((uint8_t)(n >> (8 * i)));
    }
    s.insert(s.end(), d, d + n);
}

// FindAndDelete (interpreter.cpp:253-279): remove every op-aligned occurrence of b.
int find_and_delete(Bytes& script, const Bytes& b) {
    int found = 0;
    if (b.empty()) return 0;
    Bytes result;
    size_t pc = 0, pc2 = 0, end = script.size();
    uint8_t op;
    do {
        result.insert(result.end(), script.begin() + pc2, script.begin() + pc);
        while (end - pc >= b.size() && memcmp(script.data() + pc, b.data(), b.size()) == 0) {
            pc += b.size();
            ++found;
        }
        pc2 = pc;
    } while (script_get_op(script.data(), script.size(), pc, op, nullptr, nullptr));
    if (found > 0) {
        result.insert(result.end(), script.begin() + pc2, script.end());
        script.swap(result);
    }
    return found;
}

// ConditionStack (interpreter.cpp:282-343)
struct CondStack {
    uint32_t size = 0, first_false = UINT32_MAX;
    bool empty() const { return size == 0; }
    bool all_true() const { return first_false == UINT32_MAX; }
    void push(bool f) {
        if (first_false == UINT32_MAX && !f) first_false = size;
        ++size;
    }
    void pop() {
        --size;
        if (first_false == size) first_false = UINT32_MAX;
    }
    void toggle_top() {
        if (first_false == UINT32_MAX) first_false = size - 1;
        else if (first_false == size - 1) first_false = UINT32_MAX;
    }
};

bool is_push_only(const Span& s) {
    size_t pc = 0;
    uint8_t op;
    while (pc < s.n) {
        if (!script_get_op(s.p, s.n, pc, op, nullptr, nullptr)) return false;
        if (op > OP_16) return false;
    }
    return true;
}

bool is_p2sh(const Span& s) {
    return s.n == 23 && s.p[0] == OP_HASH160 && s.p[1] == 0x14 && s.p[22] == OP_EQUAL;
}

// CScript::IsWitnessProgram (script.cpp:218-233)
bool is_witness_program(const uint8_t* p, size_t n, int& version, Bytes& program) {
    if (n < 4 || n > 42) return false;
    if (p[0] != OP_0 && (p[0] < OP_1 || p[0] > OP_16)) return false;
    if ((size_t)p[1] + 2 == n) {
        version = p[0] == OP_0 ? 0 : (int)p[0] - (int)(OP_1 - 1);
        program.assign(p + 2, p + n);
        return true;
    }
    return false;
}

#define STACKTOP(i) (stack.at(stack.size() + (i)))

void popstack(std::vector<Bytes>& st) {
    if (st.empty()) throw std::runtime_error("popstack(): stack empty");
    st.pop_back();
}

bool eval_script(std::vector<Bytes>& stack, const uint8_t* script, size_t script_len,
                 unsigned flags, SigChecker& checker, SigVersion sigversion, ScriptErr* serror) {
    static const Bytes vch_false;
    static const Bytes vch_true(1, 1);
    if (serror) *serror = SERR_UNKNOWN;
    if (script_len > MAX_SCRIPT_SIZE) return fail(serror, SERR_SCRIPT_SIZE);
    size_t pc = 0, pbegincodehash = 0;
    const size_t pend = script_len;
    CondStack vf_exec;
    std::vector<Bytes> altstack;
    int op_count = 0;
    try {
        while (pc < pend) {
            bool f_exec = vf_exec.all_true();
            uint8_t opcode;
            const uint8_t* pdata = nullptr;
            size_t plen = 0;
            if (!script_get_op(script, script_len, pc, opcode, &pdata, &plen))
                return fail(serror, SERR_BAD_OPCODE);
            if (plen > MAX_SCRIPT_ELEMENT_SIZE) return fail(serror, SERR_PUSH_SIZE);
            if (opcode > OP_16 && ++op_count > MAX_OPS_PER_SCRIPT) return fail(serror, SERR_OP_COUNT);
            switch (opcode) {  // disabled opcodes fail even when not executed (CVE-2010-5137)
                case OP_CAT: case OP_SUBSTR: case OP_LEFT: case OP_RIGHT: case OP_INVERT:
                case OP_AND: case OP_OR: case OP_XOR: case OP_2MUL: case OP_2DIV: case OP_MUL:
                case OP_DIV: case OP_MOD: case OP_LSHIFT: case OP_RSHIFT:
                    return fail(serror, SERR_DISABLED_OPCODE);
                default:
                    break;
            }
            if (f_exec && opcode <= OP_PUSHDATA4) {
                stack.emplace_back(pdata, pdata + plen);
            } else if (f_exec || (OP_IF <= opcode && opcode <= OP_ENDIF)) {
                switch (opcode) {
                    case OP_1NEGATE:
                    case 0x51: case 0x52: case 0x53: case 0x54: case 0x55: case 0x56: case 0x57:
                    case 0x58: case 0x59: case 0x5a: case 0x5b: case 0x5c: case 0x5d: case 0x5e:
                    case 0x5f: case 0x60:
                        stack.push_back(num_encode((int)opcode - (int)(OP_1 - 1)));
                        break;
                    case OP_NOP:
                        break;
                    case OP_CHECKLOCKTIMEVERIFY: {
                        if (!(flags & FLAG_CHECKLOCKTIMEVERIFY)) break;  // NOP2
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int64_t lt = num_decode(STACKTOP(-1), 5);
                        if (lt < 0) return fail(serror, SERR_NEGATIVE_LOCKTIME);
                        if (!checker.check_locktime(lt)) return fail(serror, SERR_UNSATISFIED_LOCKTIME);
                        break;
                    }
                    case OP_CHECKSEQUENCEVERIFY: {
                        if (!(flags & FLAG_CHECKSEQUENCEVERIFY)) break;  // NOP3
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int64_t sq = num_decode(STACKTOP(-1), 5);
                        if (sq < 0) return fail(serror, SERR_NEGATIVE_LOCKTIME);
                        if ((sq & (int64_t)SEQUENCE_LOCKTIME_DISABLE_FLAG) != 0) break;
                        if (!checker.check_sequence(sq)) return fail(serror, SERR_UNSATISFIED_LOCKTIME);
                        break;
                    }
                    case OP_NOP1: case 0xb3: case 0xb4: case 0xb5: case 0xb6: case 0xb7: case 0xb8:
                    case 0xb9:
                        break;  // DISCOURAGE_UPGRADABLE_NOPS is not a libconsensus flag
                    case OP_IF:
                    case OP_NOTIF: {
                        bool value = false;
                        if (f_exec) {
                            if (stack.size() < 1) return fail(serror, SERR_UNBALANCED_CONDITIONAL);
                            value = cast_to_bool(STACKTOP(-1));
                            if (opcode == OP_NOTIF) value = !value;
                            popstack(stack);
                        }
                        vf_exec.push(value);
                        break;
                    }
                    case OP_ELSE:
                        if (vf_exec.empty()) return fail(serror, SERR_UNBALANCED_CONDITIONAL);
                        vf_exec.toggle_top();
                        break;
                    case OP_ENDIF:
                        if (vf_exec.empty()) return fail(serror, SERR_UNBALANCED_CONDITIONAL);
                        vf_exec.pop();
                        break;
                    case OP_VERIFY: {
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        if (cast_to_bool(STACKTOP(-1))) popstack(stack);
                        else return fail(serror, SERR_VERIFY);
                        break;
                    }
                    case OP_RETURN:
                        return fail(serror, SERR_OP_RETURN);
                    case OP_TOALTSTACK:
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        altstack.push_back(STACKTOP(-1));
                        popstack(stack);
                        break;
                    case OP_FROMALTSTACK:
                        if (altstack.size() < 1) return fail(serror, SERR_INVALID_ALTSTACK_OPERATION);
                        stack.push_back(altstack.back());
                        popstack(altstack);
                        break;
                    case OP_2DROP:
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        popstack(stack);
                        popstack(stack);
                        break;
                    case OP_2DUP: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes a = STACKTOP(-2), b = STACKTOP(-1);
                        stack.push_back(a);
                        stack.push_back(b);
                        break;
                    }
                    case OP_3DUP: {
                        if (stack.size() < 3) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes a = STACKTOP(-3), b = STACKTOP(-2), c = STACKTOP(-1);
                        stack.push_back(a);
                        stack.push_back(b);
                        stack.push_back(c);
                        break;
                    }
                    case OP_2OVER: {
                        if (stack.size() < 4) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes a = STACKTOP(-4), b = STACKTOP(-3);
                        stack.push_back(a);
                        stack.push_back(b);
                        break;
                    }
                    case OP_2ROT: {
                        if (stack.size() < 6) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes a = STACKTOP(-6), b = STACKTOP(-5);
                        stack.erase(stack.end() - 6, stack.end() - 4);
                        stack.push_back(a);
                        stack.push_back(b);
                        break;
                    }
                    case OP_2SWAP:
                        if (stack.size() < 4) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        std::swap(STACKTOP(-4), STACKTOP(-2));
                        std::swap(STACKTOP(-3), STACKTOP(-1));
                        break;
                    case OP_IFDUP: {
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes v = STACKTOP(-1);
                        if (cast_to_bool(v)) stack.push_back(v);
                        break;
                    }
                    case OP_DEPTH:
                        stack.push_back(num_encode((int64_t)stack.size()));
                        break;
                    case OP_DROP:
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        popstack(stack);
                        break;
                    case OP_DUP: {
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes v = STACKTOP(-1);
                        stack.push_back(v);
                        break;
                    }
                    case OP_NIP:
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        stack.erase(stack.end() - 2);
                        break;
                    case OP_OVER: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes v = STACKTOP(-2);
                        stack.push_back(v);
                        break;
                    }
                    case OP_PICK:
                    case OP_ROLL: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int n = num_getint(num_decode(STACKTOP(-1)));
                        popstack(stack);
                        if (n < 0 || n >= (int)stack.size())
                            return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes v = STACKTOP(-n - 1);
                        if (opcode == OP_ROLL) stack.erase(stack.end() - n - 1);
                        stack.push_back(v);
                        break;
                    }
                    case OP_ROT:
                        if (stack.size() < 3) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        std::swap(STACKTOP(-3), STACKTOP(-2));
                        std::swap(STACKTOP(-2), STACKTOP(-1));
                        break;
                    case OP_SWAP:
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        std::swap(STACKTOP(-2), STACKTOP(-1));
                        break;
                    case OP_TUCK: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes v = STACKTOP(-1);
                        stack.insert(stack.end() - 2, v);
                        break;
                    }
                    case OP_SIZE:
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        stack.push_back(num_encode((int64_t)STACKTOP(-1).size()));
                        break;
                    case OP_EQUAL:
                    case OP_EQUALVERIFY: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        bool eq = STACKTOP(-2) == STACKTOP(-1);
                        popstack(stack);
                        popstack(stack);
                        stack.push_back(eq ? vch_true : vch_false);
                        if (opcode == OP_EQUALVERIFY) {
                            if (eq) popstack(stack);
                            else return fail(serror, SERR_EQUALVERIFY);
                        }
                        break;
                    }
                    case OP_1ADD: case OP_1SUB: case OP_NEGATE: case OP_ABS: case OP_NOT:
                    case OP_0NOTEQUAL: {
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int64_t bn = num_decode(STACKTOP(-1));
                        switch (opcode) {
                            case OP_1ADD: bn += 1; break;
                            case OP_1SUB: bn -= 1; break;
                            case OP_NEGATE: bn = -bn; break;
                            case OP_ABS: if (bn < 0) bn = -bn; break;
                            case OP_NOT: bn = (bn == 0); break;
                            default: bn = (bn != 0); break;
                        }
                        popstack(stack);
                        stack.push_back(num_encode(bn));
                        break;
                    }
                    case OP_ADD: case OP_SUB: case OP_BOOLAND: case OP_BOOLOR: case OP_NUMEQUAL:
                    case OP_NUMEQUALVERIFY: case OP_NUMNOTEQUAL: case OP_LESSTHAN:
                    case OP_GREATERTHAN: case OP_LESSTHANOREQUAL: case OP_GREATERTHANOREQUAL:
                    case OP_MIN: case OP_MAX: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int64_t a = num_decode(STACKTOP(-2)), b = num_decode(STACKTOP(-1)), r = 0;
                        switch (opcode) {
                            case OP_ADD: r = a + b; break;
                            case OP_SUB: r = a - b; break;
                            case OP_BOOLAND: r = (a != 0 && b != 0); break;
                            case OP_BOOLOR: r = (a != 0 || b != 0); break;
                            case OP_NUMEQUAL: case OP_NUMEQUALVERIFY: r = (a == b); break;
                            case OP_NUMNOTEQUAL: r = (a != b); break;
                            case OP_LESSTHAN: r = (a < b); break;
                            case OP_GREATERTHAN: r = (a > b); break;
                            case OP_LESSTHANOREQUAL: r = (a <= b); break;
                            case OP_GREATERTHANOREQUAL: r = (a >= b); break;
                            case OP_MIN: r = a < b ? a : b; break;
                            default: r = a > b ? a : b; break;
                        }
                        popstack(stack);
                        popstack(stack);
                        stack.push_back(num_encode(r));
                        if (opcode == OP_NUMEQUALVERIFY) {
                            if (cast_to_bool(STACKTOP(-1))) popstack(stack);
                            else return fail(serror, SERR_NUMEQUALVERIFY);
                        }
                        break;
                    }
                    case OP_WITHIN: {
                        if (stack.size() < 3) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int64_t x = num_decode(STACKTOP(-3)), lo = num_decode(STACKTOP(-2)),
                                hi = num_decode(STACKTOP(-1));
                        bool v = lo <= x && x < hi;
                        popstack(stack);
                        popstack(stack);
                        popstack(stack);
                        stack.push_back(v ? vch_true : vch_false);
                        break;
                    }
                    case OP_RIPEMD160: case OP_SHA1: case OP_SHA256: case OP_HASH160:
                    case OP_HASH256: {
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        const Bytes& v = STACKTOP(-1);
                        Bytes h((opcode == OP_RIPEMD160 || opcode == OP_SHA1 || opcode == OP_HASH160) ? 20 : 32);
                        if (opcode == OP_RIPEMD160) ripemd160(v.data(), v.size(), h.data());
                        else if (opcode == OP_SHA1) sha1(v.data(), v.size(), h.data());
                        else if (opcode == OP_SHA256) sha256(v.data(), v.size(), h.data());
                        else if (opcode == OP_HASH160) {
                            const uint8_t* c = checker.cached_hash160(v.data(), v.size());
                            if (c) memcpy(h.data(), c, 20);
                            else hash160(v.data(), v.size(), h.data());
                        }
                        else sha256d(v.data(), v.size(), h.data());
                        popstack(stack);
                        stack.push_back(std::move(h));
                        break;
                    }
                    case OP_CODESEPARATOR:
                        pbegincodehash = pc;
                        break;
                    case OP_CHECKSIG:
                    case OP_CHECKSIGVERIFY: {
                        if (stack.size() < 2) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        const Bytes& sig = STACKTOP(-2);
                        const Bytes& pub = STACKTOP(-1);
                        // EvalChecksigPreTapscript (interpreter.cpp:345-369)
                        Bytes code(script + pbegincodehash, script + pend);
                        if (sigversion == SIGVERSION_BASE) {
                            Bytes pushed;
                            push_data(pushed, sig.data(), sig.size());
                            find_and_delete(code, pushed);
                        }
                        if (!sig.empty() && (flags & FLAG_DERSIG) && !is_valid_signature_encoding(sig))
                            return fail(serror, SERR_SIG_DER);
                        bool ok = checker.check_ecdsa(sig, pub, code, sigversion);
                        popstack(stack);
                        popstack(stack);
                        stack.push_back(ok ? vch_true : vch_false);
                        if (opcode == OP_CHECKSIGVERIFY) {
                            if (ok) popstack(stack);
                            else return fail(serror, SERR_CHECKSIGVERIFY);
                        }
                        break;
                    }
                    case OP_CHECKMULTISIG:
                    case OP_CHECKMULTISIGVERIFY: {
                        // interpreter.cpp:1129-1239
                        int i = 1;
                        if ((int)stack.size() < i) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int nkeys = num_getint(num_decode(STACKTOP(-i)));
                        if (nkeys < 0 || nkeys > MAX_PUBKEYS_PER_MULTISIG)
                            return fail(serror, SERR_PUBKEY_COUNT);
                        op_count += nkeys;
                        if (op_count > MAX_OPS_PER_SCRIPT) return fail(serror, SERR_OP_COUNT);
                        int ikey = ++i;
                        i += nkeys;
                        if ((int)stack.size() < i) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        int nsigs = num_getint(num_decode(STACKTOP(-i)));
                        if (nsigs < 0 || nsigs > nkeys) return fail(serror, SERR_SIG_COUNT);
                        int isig = ++i;
                        i += nsigs;
                        if ((int)stack.size() < i) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        Bytes code(script + pbegincodehash, script + pend);
                        for (int k = 0; k < nsigs; k++) {
                            if (sigversion == SIGVERSION_BASE) {
                                const Bytes& sg = STACKTOP(-isig - k);
                                Bytes pushed;
                                push_data(pushed, sg.data(), sg.size());
                                find_and_delete(code, pushed);
                            }
                        }
                        // candidate pairs: sig k can only meet keys k .. k + nkeys - nsigs
                        // (the loop below never skips a signature); queue them all at once when
                        // that is at most 2 x nkeys checks (or the checker asks for all), so a
                        // batching checker needs no extra round for the key advance
                        if (nsigs > 0 && (checker.hint_all() ||
                                          (long)nsigs * (nkeys - nsigs + 1) <= 2L * nkeys)) {
                            for (int k = 0; k < nsigs; k++) {
                                const Bytes& sg = STACKTOP(-isig - k);
                                if (sg.empty() || ((flags & FLAG_DERSIG) && !is_valid_signature_encoding(sg)))
                                    continue;
                                for (int j = k; j <= k + nkeys - nsigs; j++)
                                    checker.hint_ecdsa(sg, STACKTOP(-ikey - j), code, sigversion);
                            }
                        }
                        bool success = true;
                        while (success && nsigs > 0) {
                            const Bytes& sig = STACKTOP(-isig);
                            const Bytes& pub = STACKTOP(-ikey);
                            if (!sig.empty() && (flags & FLAG_DERSIG) && !is_valid_signature_encoding(sig))
                                return fail(serror, SERR_SIG_DER);
                            bool ok = checker.check_ecdsa(sig, pub, code, sigversion);
                            if (ok) {
                                isig++;
                                nsigs--;
                            }
                            ikey++;
                            nkeys--;
                            if (nsigs > nkeys) success = false;
                        }
                        while (i-- > 1) popstack(stack);
                        if (stack.size() < 1) return fail(serror, SERR_INVALID_STACK_OPERATION);
                        if ((flags & FLAG_NULLDUMMY) && STACKTOP(-1).size())
                            return fail(serror, SERR_SIG_NULLDUMMY);
                        popstack(stack);
                        stack.push_back(success ? vch_true : vch_false);
                        if (opcode == OP_CHECKMULTISIGVERIFY) {
                            if (success) popstack(stack);
                            else return fail(serror, SERR_CHECKMULTISIGVERIFY);
                        }
                        break;
                    }
                    default:
                        return fail(serror, SERR_BAD_OPCODE);
                }
            }
            if (stack.size() + altstack.size() > MAX_STACK_SIZE) return fail(serror, SERR_STACK_SIZE);
        }
    } catch (...) {
        return fail(serror, SERR_UNKNOWN);
    }
    if (!vf_exec.empty()) return fail(serror, SERR_UNBALANCED_CONDITIONAL);
    if (serror) *serror = SERR_OK;
    return true;
}

// eval_script of a P2PKH scriptPubKey (DUP HASH160 <20> EQUALVERIFY CHECKSIG, SIGVERSION_BASE) on
// a stack of 2..100 elements, unrolled: the same checks in the same order with the same errors and
// the same resulting stack.  With that depth none of eval_script's size / op-count / stack limits
// can trip, and the script has no OP_CODESEPARATOR, so the scriptCode is the whole script (after
// FindAndDelete of the signature push, as for any BASE CHECKSIG).  Returns false when the shape
// does not apply (the caller then runs eval_script); *res holds eval_script's result otherwise.
// HASH160(key) == prog20 (the checker's batched hash when it holds one)
bool key_hash_equal(SigChecker& checker, const uint8_t* key, size_t n, const uint8_t* prog20) {
    uint8_t h[20];
    const uint8_t* hk = checker.cached_hash160(key, n);
    if (!hk) {
        hash160(key, n, h);
        hk = h;
    }
    return memcmp(hk, prog20, 20) == 0;
}

bool eval_p2pkh(std::vector<Bytes>& stack, const Span& spk, unsigned flags, SigChecker& checker,
                ScriptErr* serror, bool* res) {
    const uint8_t* s = spk.p;
    if (spk.n != 25 || s[0] != OP_DUP || s[1] != OP_HASH160 || s[2] != 0x14 ||
        s[23] != OP_EQUALVERIFY || s[24] != OP_CHECKSIG)
        return false;
    if (stack.size() < 2 || stack.size() > 100) return false;
    static const Bytes vch_false;
    static const Bytes vch_true(1, 1);
    const Bytes& sig = stack[stack.size() - 2];
    const Bytes& pub = stack[stack.size() - 1];
    const bool der_bad = !sig.empty() && (flags & FLAG_DERSIG) && !is_valid_signature_encoding(sig);
    // OP_DUP, OP_HASH160, <20> OP_EQUALVERIFY: taken over by the checker when the run goes on to
    // the signature check (no DER failure in between), else compared here
    const bool taken = !der_bad && checker.defer_key_hash(pub.data(), pub.size(), s + 3);
    if (!taken && !key_hash_equal(checker, pub.data(), pub.size(), s + 3)) {
        *res = fail(serror, SERR_EQUALVERIFY);
        return true;
    }
    if (der_bad) {
        *res = fail(serror, SERR_SIG_DER);
        return true;
    }
    Bytes code(s, s + 25);  // OP_CHECKSIG (EvalChecksigPreTapscript, interpreter.cpp:345-369)
    Bytes pushed;
    push_data(pushed, sig.data(), sig.size());
    find_and_delete(code, pushed);
    const bool ok = checker.check_ecdsa(sig, pub, code, SIGVERSION_BASE);
    if (taken && !checker.key_hash_taken() && !key_hash_equal(checker, pub.data(), pub.size(), s + 3)) {
        *res = fail(serror, SERR_EQUALVERIFY);
        return true;
    }
    popstack(stack);
    popstack(stack);
    stack.push_back(ok ? vch_true : vch_false);
    if (serror) *serror = SERR_OK;
    *res = true;
    return true;
}

bool execute_witness_script(std::vector<Bytes> stack, const uint8_t* script, size_t len,
                            unsigned flags, SigChecker& checker, ScriptErr* serror) {
    for (const auto& e : stack)
        if (e.size() > MAX_SCRIPT_ELEMENT_SIZE) return fail(serror, SERR_PUSH_SIZE);
    if (!eval_script(stack, script, len, flags, checker, SIGVERSION_WITNESS_V0, serror)) return false;
    if (stack.size() != 1) return fail(serror, SERR_CLEANSTACK);
    if (!cast_to_bool(stack.back())) return fail(serror, SERR_EVAL_FALSE);
    return true;
}

bool verify_witness_program(const std::vector<Span>& witness, int version, const Span& program,
                            unsigned flags, SigChecker& checker, ScriptErr* serror) {
    if (version == 0) {
        if (program.n == 32) {  // P2WSH
            if (witness.empty()) return fail(serror, SERR_WITNESS_PROGRAM_WITNESS_EMPTY);
            const Span& sc = witness.back();
            uint8_t h[32];
            sha256(sc.p, sc.n, h);
            if (memcmp(h, program.p, 32) != 0) return fail(serror, SERR_WITNESS_PROGRAM_MISMATCH);
            std::vector<Bytes> stack;
            stack.reserve(witness.size() + 4);  // no regrowth in the common scripts
            for (size_t k = 0; k + 1 < witness.size(); k++)
                stack.emplace_back(witness[k].p, witness[k].p + witness[k].n);
            return execute_witness_script(std::move(stack), sc.p, sc.n, flags, checker, serror);
        } else if (program.n == 20) {  // P2WPKH: DUP HASH160 <20> EQUALVERIFY CHECKSIG
            if (witness.size() != 2) return fail(serror, SERR_WITNESS_PROGRAM_MISMATCH);
            uint8_t sc[25] = {OP_DUP, OP_HASH160, 0x14};
            memcpy(sc + 3, program.p, 20);
            sc[23] = OP_EQUALVERIFY;
            sc[24] = OP_CHECKSIG;
            // execute_witness_script on [sig, key] with this script, unrolled: the same checks in
            // the same order with the same errors (none of eval_script's size / op-count / stack
            // limits can trip on this script and a two-element stack)
            for (const auto& w : witness)
                if (w.n > MAX_SCRIPT_ELEMENT_SIZE) return fail(serror, SERR_PUSH_SIZE);
            const Span& ws = witness[0];
            const Span& wk = witness[1];
            const Bytes sig(ws.p, ws.p + ws.n);
            const bool der_bad = !sig.empty() && (flags & FLAG_DERSIG) && !is_valid_signature_encoding(sig);
            // OP_DUP, OP_HASH160, <20> OP_EQUALVERIFY: taken over by the checker when the run goes
            // on to the signature check, else compared here
            const bool taken = !der_bad && checker.defer_key_hash(wk.p, wk.n, program.p);
            if (!taken && !key_hash_equal(checker, wk.p, wk.n, program.p))
                return fail(serror, SERR_EQUALVERIFY);
            // OP_CHECKSIG (witness v0: no FindAndDelete; scriptCode = the whole script)
            if (der_bad) return fail(serror, SERR_SIG_DER);
            const Bytes pub(wk.p, wk.p + wk.n), code(sc, sc + 25);
            const bool ok = checker.check_ecdsa(sig, pub, code, SIGVERSION_WITNESS_V0);
            if (taken && !checker.key_hash_taken() && !key_hash_equal(checker, wk.p, wk.n, program.p))
                return fail(serror, SERR_EQUALVERIFY);
            // the stack is [result]: clean; false -> EVAL_FALSE
            if (!ok) return fail(serror, SERR_EVAL_FALSE);
            if (serror) *serror = SERR_OK;
            return true;
        }
        return fail(serror, SERR_WITNESS_PROGRAM_WRONG_LENGTH);
    }
    // witness v1+ : SCRIPT_VERIFY_TAPROOT is not a libconsensus flag -> succeed unchecked
    // (interpreter.cpp:1885-1887, :1927-1932)
    return true;
}

}  // namespace

bool script_get_op(const uint8_t* s, size_t n, size_t& pc, uint8_t& op, const uint8_t** data,
                   size_t* datalen) {
    if (data) *data = nullptr;
    if (datalen) *datalen = 0;
    if (pc >= n) return false;
    uint8_t o = s[pc++];
    op = 0xff;
    if (o <= OP_PUSHDATA4) {
        size_t sz;
        if (o < OP_PUSHDATA1) {
            sz = o;
        } else if (o == OP_PUSHDATA1) {
            if (n - pc < 1) return false;
            sz = s[pc];
            pc += 1;
        } else if (o == OP_PUSHDATA2) {
            if (n - pc < 2) return false;
            sz = (size_t)s[pc] | ((size_t)s[pc + 1] << 8);
            pc += 2;
        } else {
            if (n - pc < 4) return false;
            sz = (size_t)s[pc] | ((size_t)s[pc + 1] << 8) | ((size_t)s[pc + 2] << 16) |
                 ((size_t)s[pc + 3] << 24);
            pc += 4;
        }
        if (n - pc < sz) return false;
        if (data) *data = s + pc;
        if (datalen) *datalen = sz;
        pc += sz;
    }
    op = o;
    return true;
}

bool is_valid_signature_encoding(const Bytes& sig) {
    if (sig.size() < 9 || sig.size() > 73) return false;
    if (sig[0] != 0x30) return false;
    if (sig[1] != sig.size() - 3) return false;
    unsigned lenR = sig[3];
    if (5 + lenR >= sig.size()) return false;
    unsigned lenS = sig[5 + lenR];
    if ((size_t)(lenR + lenS + 7) != sig.size()) return false;
    if (sig[2] != 0x02) return false;
    if (lenR == 0) return false;
    if (sig[4] & 0x80) return false;
    if (lenR > 1 && sig[4] == 0x00 && !(sig[5] & 0x80)) return false;
    if (sig[lenR + 4] != 0x02) return false;
    if (lenS == 0) return false;
    if (sig[lenR + 6] & 0x80) return false;
    if (lenS > 1 && sig[lenR + 6] == 0x00 && !(sig[lenR + 7] & 0x80)) return false;
    return true;
}

bool tx_check_locktime(const Tx& tx, unsigned nin, int64_t lt) {
    int64_t txlt = (int64_t)tx.locktime;
    if (!((txlt < LOCKTIME_THRESHOLD && lt < LOCKTIME_THRESHOLD) ||
          (txlt >= LOCKTIME_THRESHOLD && lt >= LOCKTIME_THRESHOLD)))
        return false;
    if (lt > txlt) return false;
    if (tx.vin[nin].sequence == SEQUENCE_FINAL) return false;
    return true;
}

bool tx_check_sequence(const Tx& tx, unsigned nin, int64_t sq) {
    const int64_t txseq = (int64_t)tx.vin[nin].sequence;
    if ((uint32_t)tx.version < 2) return false;
    if (txseq & SEQUENCE_LOCKTIME_DISABLE_FLAG) return false;
    const int64_t mask = SEQUENCE_LOCKTIME_TYPE_FLAG | SEQUENCE_LOCKTIME_MASK;
    const int64_t a = txseq & mask, b = sq & mask;
    if (!((a < SEQUENCE_LOCKTIME_TYPE_FLAG && b < SEQUENCE_LOCKTIME_TYPE_FLAG) ||
          (a >= SEQUENCE_LOCKTIME_TYPE_FLAG && b >= SEQUENCE_LOCKTIME_TYPE_FLAG)))
        return false;
    if (b > a) return false;
    return true;
}

bool verify_script(const Span& script_sig, const Span& spk, const std::vector<Span>& witness,
                   unsigned flags, SigChecker& checker, ScriptErr* serror) {
    if (serror) *serror = SERR_UNKNOWN;
    // Native P2WPKH with an empty scriptSig: the general path below evaluates nothing, then pushes
    // OP_0 and the 20-byte program (no error is possible), tests the program with CastToBool,
    // finds a v0 program and runs it; P2SH does not apply.  The same steps without the stacks.
    if ((flags & FLAG_WITNESS) && script_sig.n == 0 && spk.n == 22 && spk.p[0] == 0 &&
        spk.p[1] == 0x14) {
        const Span prog{spk.p + 2, 20};
        if (!cast_to_bool(prog.p, prog.n)) return fail(serror, SERR_EVAL_FALSE);
        if (!verify_witness_program(witness, 0, prog, flags, checker, serror)) return false;
        if (serror) *serror = SERR_OK;
        return true;
    }
    bool had_witness = false;
    std::vector<Bytes> stack, stack_copy;
    stack.reserve(8);
    if (!eval_script(stack, script_sig.p, script_sig.n, flags, checker, SIGVERSION_BASE, serror))
        return false;
    if (flags & FLAG_P2SH) stack_copy = stack;
    bool spk_ok;
    if (!eval_p2pkh(stack, spk, flags, checker, serror, &spk_ok))
        spk_ok = eval_script(stack, spk.p, spk.n, flags, checker, SIGVERSION_BASE, serror);
    if (!spk_ok) return false;
    if (stack.empty() || !cast_to_bool(stack.back())) return fail(serror, SERR_EVAL_FALSE);

    int wv;
    Bytes wp;
    if ((flags & FLAG_WITNESS) && is_witness_program(spk.p, spk.n, wv, wp)) {
        had_witness = true;
        if (script_sig.n != 0) return fail(serror, SERR_WITNESS_MALLEATED);
        if (!verify_witness_program(witness, wv, Span{wp.data(), wp.size()}, flags, checker, serror))
            return false;
        stack.resize(1);
    }

    if ((flags & FLAG_P2SH) && is_p2sh(spk)) {
        if (!is_push_only(script_sig)) return fail(serror, SERR_SIG_PUSHONLY);
        stack.swap(stack_copy);
        Bytes redeem = stack.back();
        popstack(stack);
        if (!eval_script(stack, redeem.data(), redeem.size(), flags, checker, SIGVERSION_BASE, serror))
            return false;
        if (stack.empty() || !cast_to_bool(stack.back())) return fail(serror, SERR_EVAL_FALSE);
        if ((flags & FLAG_WITNESS) && is_witness_program(redeem.data(), redeem.size(), wv, wp)) {
            had_witness = true;
            Bytes expect;
            push_data(expect, redeem.data(), redeem.size());
            if (script_sig.n != expect.size() || memcmp(script_sig.p, expect.data(), expect.size()) != 0)
                return fail(serror, SERR_WITNESS_MALLEATED_P2SH);
            if (!verify_witness_program(witness, wv, Span{wp.data(), wp.size()}, flags, checker, serror))
                return false;
            stack.resize(1);
        }
    }
    // CLEANSTACK is not a libconsensus flag.
    if (flags & FLAG_WITNESS) {
        // (the reference asserts P2SH here; see DESIGN.md "divergences")
        if (!had_witness && !witness.empty()) return fail(serror, SERR_WITNESS_UNEXPECTED);
    }
    if (serror) *serror = SERR_OK;
    return true;
}

}  // namespace host
}  // namespace bcc
