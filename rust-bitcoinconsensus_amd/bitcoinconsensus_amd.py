"""Python mirror of rust-bitcoinconsensus's API (src/lib.rs) over the engine's C ABI.

This is the host-side surface a user of the reference crate switches to:

    verify(spent_output, amount, spending_transaction, input_index)      src/lib.rs:103-110
    verify_with_flags(..., flags)                                        src/lib.rs:113-139
    height_to_flags(height), version()                                   src/lib.rs:45-68
    VERIFY_* constants, Error enum                                       src/lib.rs:22-42, 164-185
    verify_batch([...])  -- new: N independent verify() calls, signature work on the GPU

plus the inner tuple ABI ``ecdsa_verify_tuples`` and device-pointer entry points
used by bench.py.  Every call goes to librbc_amd.so (HIP kernels for gfx950); if the library is
missing the import fails loudly — there is no CPU fallback.
"""
import ctypes
import enum
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librbc_amd.so")

VERIFY_NONE = 0
VERIFY_P2SH = 1 << 0
VERIFY_DERSIG = 1 << 2
VERIFY_NULLDUMMY = 1 << 4
VERIFY_CHECKLOCKTIMEVERIFY = 1 << 9
VERIFY_CHECKSEQUENCEVERIFY = 1 << 10
VERIFY_WITNESS = 1 << 11
VERIFY_ALL = (VERIFY_P2SH | VERIFY_DERSIG | VERIFY_NULLDUMMY | VERIFY_CHECKLOCKTIMEVERIFY
              | VERIFY_CHECKSEQUENCEVERIFY | VERIFY_WITNESS)


class Error(enum.IntEnum):
    """Mirrors the Rust ``Error`` (repr(C)); ERR_SCRIPT = 0 doubles as C's ERR_OK."""
    ERR_SCRIPT = 0
    ERR_TX_INDEX = 1
    ERR_TX_SIZE_MISMATCH = 2
    ERR_TX_DESERIALIZE = 3
    ERR_AMOUNT_REQUIRED = 4
    ERR_INVALID_FLAGS = 5


class ConsensusError(Exception):
    def __init__(self, err):
        super().__init__(err.name)
        self.error = err


_lib = None


def lib():
    """Load librbc_amd.so (raises if it has not been built: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: build with `make -C {_HERE}` "
                              "(or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        u8p, sz = ctypes.c_char_p, ctypes.c_size_t
        vp = ctypes.c_void_p
        L.mi_ecdsa_verify_tuples.argtypes = [u8p, u8p, u8p, u8p, u8p, sz, ctypes.c_int]
        L.mi_ecdsa_verify_device.argtypes = [vp] * 7 + [sz, vp]
        L.mi_microbench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        _lib = L
    return _lib


def height_to_flags(height):
    """Soft-fork activation heights (src/lib.rs:45-65)."""
    flag = VERIFY_NONE
    if height >= 173805:
        flag |= VERIFY_P2SH
    if height >= 363725:
        flag |= VERIFY_DERSIG
    if height >= 388381:
        flag |= VERIFY_CHECKLOCKTIMEVERIFY
    if height >= 419328:
        flag |= VERIFY_CHECKSEQUENCEVERIFY
    if height >= 481824:
        flag |= VERIFY_NULLDUMMY | VERIFY_WITNESS
    return flag


def ecdsa_verify_tuples(pub65, msg32, r32, s32, device=0):
    """Inner tuple ABI: n tuples as concatenated byte strings -> bytes of verdicts (0/1)."""
    n = len(msg32) // 32
    assert len(pub65) == 65 * n and len(r32) == 32 * n and len(s32) == 32 * n
    out = ctypes.create_string_buffer(max(n, 1))
    rc = lib().mi_ecdsa_verify_tuples(pub65, msg32, r32, s32, out, n, device)
    if rc != 0:
        raise RuntimeError(f"mi_ecdsa_verify_tuples failed: hip error {rc}")
    return out.raw[:n]


def microbench(op, iters=4096):
    r = ctypes.c_double(0)
    rc = lib().mi_microbench(op, iters, ctypes.byref(r))
    if rc != 0:
        raise RuntimeError(f"mi_microbench failed: {rc}")
    return r.value
