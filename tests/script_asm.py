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
