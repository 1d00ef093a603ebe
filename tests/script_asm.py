"""Test helpers: Bitcoin script asm parsing and the script_tests transaction construction.

* ``parse_script`` restates ParseScript (depend/bitcoin/src/core_read.cpp:24-93): decimal numbers
  are pushed as script numbers (OP_0 / OP_1NEGATE / OP_1..16 / minimal CScriptNum push), ``0x..``
  is inserted raw, ``'str'`` is pushed, opcode names are accepted with or without ``OP_``.
* ``crediting_tx`` / ``spending_tx`` restate BuildCreditingTransaction / BuildSpendingTransaction
  (depend/bitcoin/src/test/util/transaction_utils.cpp:9-41) used by script_tests.cpp's DoTest.
* ``parse_flags`` restates ParseScriptFlags (test/transaction_tests.cpp:41-80).
"""
import hashlib
import struct

OPCODES = {
    "OP_PUSHDATA1": 0x4c, "OP_PUSHDATA2": 0x4d, "OP_PUSHDATA4": 0x4e, "OP_RESERVED": 0x50,
    "OP_NOP": 0x61, "OP_VER": 0x62, "OP_IF": 0x63, "OP_NOTIF": 0x64, "OP_VERIF": 0x65,
    "OP_VERNOTIF": 0x66, "OP_ELSE": 0x67, "OP_ENDIF": 0x68, "OP_VERIFY": 0x69, "OP_RETURN": 0x6a,
    "OP_TOALTSTACK": 0x6b, "OP_FROMALTSTACK": 0x6c, "OP_2DROP": 0x6d, "OP_2DUP": 0x6e,
    "OP_3DUP": 0x6f, "OP_2OVER": 0x70, "OP_2ROT": 0x71, "OP_2SWAP": 0x72, "OP_IFDUP": 0x73,
    "OP_DEPTH": 0x74, "OP_DROP": 0x75, "OP_DUP": 0x76, "OP_NIP": 0x77, "OP_OVER": 0x78,
    "OP_PICK": 0x79, "OP_ROLL": 0x7a, "OP_ROT": 0x7b, "OP_SWAP": 0x7c, "OP_TUCK": 0x7d,
    "OP_CAT": 0x7e, "OP_SUBSTR": 0x7f, "OP_LEFT": 0x80, "OP_RIGHT": 0x81, "OP_SIZE": 0x82,
    "OP_INVERT": 0x83, "OP_AND": 0x84, "OP_OR": 0x85, "OP_XOR": 0x86, "OP_EQUAL": 0x87,
    "OP_EQUALVERIFY": 0x88, "OP_RESERVED1": 0x89, "OP_RESERVED2": 0x8a, "OP_1ADD": 0x8b,
    "OP_1SUB": 0x8c, "OP_2MUL": 0x8d, "OP_2DIV": 0x8e, "OP_NEGATE": 0x8f, "OP_ABS": 0x90,
    "OP_NOT": 0x91, "OP_0NOTEQUAL": 0x92, "OP_ADD": 0x93, "OP_SUB": 0x94, "OP_MUL": 0x95,
    "OP_DIV": 0x96, "OP_MOD": 0x97, "OP_LSHIFT": 0x98, "OP_RSHIFT": 0x99, "OP_BOOLAND": 0x9a,
    "OP_BOOLOR": 0x9b, "OP_NUMEQUAL": 0x9c, "OP_NUMEQUALVERIFY": 0x9d, "OP_NUMNOTEQUAL": 0x9e,
    "OP_LESSTHAN": 0x9f, "OP_GREATERTHAN": 0xa0, "OP_LESSTHANOREQUAL": 0xa1,
    "OP_GREATERTHANOREQUAL": 0xa2, "OP_MIN": 0xa3, "OP_MAX": 0xa4, "OP_WITHIN": 0xa5,
    "OP_RIPEMD160": 0xa6, "OP_SHA1": 0xa7, "OP_SHA256": 0xa8, "OP_HASH160": 0xa9,
    "OP_HASH256": 0xaa, "OP_CODESEPARATOR": 0xab, "OP_CHECKSIG": 0xac, "OP_CHECKSIGVERIFY": 0xad,
    "OP_CHECKMULTISIG": 0xae, "OP_CHECKMULTISIGVERIFY": 0xaf, "OP_NOP1": 0xb0,
    "OP_CHECKLOCKTIMEVERIFY": 0xb1, "OP_CHECKSEQUENCEVERIFY": 0xb2, "OP_NOP4": 0xb3,
    "OP_NOP5": 0xb4, "OP_NOP6": 0xb5, "OP_NOP7": 0xb6, "OP_NOP8": 0xb7, "OP_NOP9": 0xb8,
    "OP_NOP10": 0xb9,
}
_NAMES = dict(OPCODES)
_NAMES.update({k[3:]: v for k, v in OPCODES.items()})

FLAG_NAMES = {"NONE": 0, "P2SH": 1 << 0, "STRICTENC": 1 << 1, "DERSIG": 1 << 2, "LOW_S": 1 << 3,
              "NULLDUMMY": 1 << 4, "SIGPUSHONLY": 1 << 5, "MINIMALDATA": 1 << 6,
              "DISCOURAGE_UPGRADABLE_NOPS": 1 << 7, "CLEANSTACK": 1 << 8,
              "CHECKLOCKTIMEVERIFY": 1 << 9, "CHECKSEQUENCEVERIFY": 1 << 10, "WITNESS": 1 << 11,
              "DISCOURAGE_UPGRADABLE_WITNESS_PROGRAM": 1 << 12, "MINIMALIF": 1 << 13,
              "NULLFAIL": 1 << 14, "WITNESS_PUBKEYTYPE": 1 << 15, "CONST_SCRIPTCODE": 1 << 16,
              "TAPROOT": 1 << 17}
VERIFY_ALL = 0xE15


def parse_flags(s):
    if not s:
        return 0
    f = 0
    for w in s.split(","):
        f |= FLAG_NAMES[w]
    return f


def scriptnum_encode(n):
    if n == 0:
        return b""
    neg = n < 0
    a = -n if neg else n
    out = bytearray()
    while a:
        out.append(a & 0xff)
        a >>= 8
    if out[-1] & 0x80:
        out.append(0x80 if neg else 0)
    elif neg:
        out[-1] |= 0x80
    return bytes(out)


def push_data(b):
    n = len(b)
    if n < 0x4c:
        return bytes([n]) + b
    if n <= 0xff:
        return b"\x4c" + bytes([n]) + b
    if n <= 0xffff:
        return b"\x4d" + struct.pack("<H", n) + b
    return b"\x4e" + struct.pack("<I", n) + b


def push_int(n):
    if n == -1 or 1 <= n <= 16:
        return bytes([n + 0x50])
    if n == 0:
        return b"\x00"
    return push_data(scriptnum_encode(n))


def parse_script(s):
    out = bytearray()
    for w in s.replace("\t", " ").replace("\n", " ").split(" "):
        if not w:
            continue
        if w.isdigit() or (w[0] == "-" and len(w) > 1 and w[1:].isdigit()):
            n = int(w)
            if n > 0xffffffff or n < -0xffffffff:
                raise ValueError("number out of range")
            out += push_int(n)
        elif w.startswith("0x") and len(w) > 2:
            out += bytes.fromhex(w[2:])
        elif len(w) >= 2 and w[0] == "'" and w[-1] == "'":
            out += push_data(w[1:-1].encode())
        elif w in _NAMES:
            out.append(_NAMES[w])
        else:
            raise ValueError("script parse error: " + w)
    return bytes(out)


def compact_size(n):
    if n < 253:
        return bytes([n])
    if n <= 0xffff:
        return b"\xfd" + struct.pack("<H", n)
    if n <= 0xffffffff:
        return b"\xfe" + struct.pack("<I", n)
    return b"\xff" + struct.pack("<Q", n)


def ser_tx(version, vin, vout, locktime, witness=None):
    """vin: [(prevout36, scriptSig, seq)], vout: [(value, script)], witness: [[bytes...] per input]"""
    has_wit = witness is not None and any(len(w) for w in witness)
    out = struct.pack("<i", version)
    if has_wit:
        out += b"\x00\x01"
    out += compact_size(len(vin))
    for po, ss, seq in vin:
        out += po + compact_size(len(ss)) + ss + struct.pack("<I", seq)
    out += compact_size(len(vout))
    for v, sc in vout:
        out += struct.pack("<q", v) + compact_size(len(sc)) + sc
    if has_wit:
        for w in witness:
            out += compact_size(len(w))
            for item in w:
                out += compact_size(len(item)) + item
    out += struct.pack("<I", locktime)
    return out


def sha256d(b):
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


def crediting_tx(spk, value):
    prevout = b"\x00" * 32 + b"\xff\xff\xff\xff"
    return ser_tx(1, [(prevout, b"\x00\x00", 0xffffffff)], [(value, spk)], 0)


def build_script_test_tx(script_sig, spk, witness, value):
    """The spending tx of DoTest: spends vout 0 of the crediting tx (txid = SHA256d of its
    non-witness serialization), value carried over, empty output script."""
    credit = crediting_tx(spk, value)
    txid = sha256d(credit)
    prevout = txid + struct.pack("<I", 0)
    return ser_tx(1, [(prevout, script_sig, 0xffffffff)], [(value, b"")], 0, [witness])


def _ripemd160(m):
    """RIPEMD-160 (Dobbertin, Bosselaers, Preneel 1996) in plain Python, for test inputs only
    (this image's hashlib has no ripemd160); pinned by the published vectors in
    tests/test_key_hash.py."""
    M = 0xFFFFFFFF
    rol = lambda x, n: ((x << n) | (x >> (32 - n))) & M  # noqa: E731
    RL = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 7, 4, 13, 1, 10, 6, 15, 3, 12, 0, 9,
          5, 2, 14, 11, 8, 3, 10, 14, 4, 9, 15, 8, 1, 2, 7, 0, 6, 13, 11, 5, 12, 1, 9, 11, 10, 0, 8,
          12, 4, 13, 3, 7, 15, 14, 5, 6, 2, 4, 0, 5, 9, 7, 12, 2, 10, 14, 1, 3, 8, 11, 6, 15, 13]
    RR = [5, 14, 7, 0, 9, 2, 11, 4, 13, 6, 15, 8, 1, 10, 3, 12, 6, 11, 3, 7, 0, 13, 5, 10, 14, 15, 8,
          12, 4, 9, 1, 2, 15, 5, 1, 3, 7, 14, 6, 9, 11, 8, 12, 2, 10, 0, 4, 13, 8, 6, 4, 1, 3, 11, 15,
          0, 5, 12, 2, 13, 9, 7, 10, 14, 12, 15, 10, 4, 1, 5, 8, 7, 6, 2, 13, 14, 0, 3, 9, 11]
    SL = [11, 14, 15, 12, 5, 8, 7, 9, 11, 13, 14, 15, 6, 7, 9, 8, 7, 6, 8, 13, 11, 9, 7, 15, 7, 12,
          15, 9, 11, 7, 13, 12, 11, 13, 6, 7, 14, 9, 13, 15, 14, 8, 13, 6, 5, 12, 7, 5, 11, 12, 14,
          15, 14, 15, 9, 8, 9, 14, 5, 6, 8, 6, 5, 12, 9, 15, 5, 11, 6, 8, 13, 12, 5, 12, 13, 14, 11,
          8, 5, 6]
    SR = [8, 9, 9, 11, 13, 15, 15, 5, 7, 7, 8, 11, 14, 14, 12, 6, 9, 13, 15, 7, 12, 8, 9, 11, 7, 7,
          12, 7, 6, 15, 13, 11, 9, 7, 15, 11, 8, 6, 6, 14, 12, 13, 5, 14, 13, 13, 7, 5, 15, 5, 8, 11,
          14, 14, 6, 14, 6, 9, 12, 9, 12, 5, 15, 8, 8, 5, 12, 9, 12, 5, 14, 6, 8, 13, 6, 5, 15, 13,
          11, 11]
    KL = [0, 0x5A827999, 0x6ED9EBA1, 0x8F1BBCDC, 0xA953FD4E]
    KR = [0x50A28BE6, 0x5C4DD124, 0x6D703EF3, 0x7A6D76E9, 0]

    def f(j, x, y, z):
        if j < 16:
            return x ^ y ^ z
        if j < 32:
            return (x & y) | (~x & z)
        if j < 48:
            return (x | ~y & M) ^ z
        if j < 64:
            return (x & z) | (y & ~z)
        return x ^ (y | ~z & M)

    h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0]
    m = m + b"\x80" + b"\x00" * ((55 - len(m)) % 64) + struct.pack("<Q", 8 * len(m))
    for o in range(0, len(m), 64):
        X = struct.unpack("<16I", m[o:o + 64])
        a1, b1, c1, d1, e1 = h
        a2, b2, c2, d2, e2 = h
        for j in range(80):
            t = (rol((a1 + (f(j, b1, c1, d1) & M) + X[RL[j]] + KL[j >> 4]) & M, SL[j]) + e1) & M
            a1, e1, d1, c1, b1 = e1, d1, rol(c1, 10), b1, t
            t = (rol((a2 + (f(79 - j, b2, c2, d2) & M) + X[RR[j]] + KR[j >> 4]) & M, SR[j]) + e2) & M
            a2, e2, d2, c2, b2 = e2, d2, rol(c2, 10), b2, t
        h = [(h[1] + c1 + d2) & M, (h[2] + d1 + e2) & M, (h[3] + e1 + a2) & M,
             (h[4] + a1 + b2) & M, (h[0] + b1 + c2) & M]
    return struct.pack("<5I", *h)


def hash160(b):
    return _ripemd160(hashlib.sha256(b).digest())
