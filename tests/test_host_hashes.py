"""CPU: the engine's host hash functions (csrc/host/hashes.cpp: SHA-256 portable and x86
SHA-extension paths, SHA-1, RIPEMD-160, HASH160) against hashlib and the published RIPEMD-160
test vectors, across message lengths that exercise every padding case."""
import ctypes
import hashlib
import os
import random
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, "native", "_build", "hash_test.so")
SRC = [os.path.join(HERE, "native", "hash_test.cpp"),
       os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc", "host", "hashes.cpp")]
DEPS = SRC + [os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc", "sha256_device.h")]

# Dobbertin-Bosselaers-Preneel, "RIPEMD-160: A Strengthened Version of RIPEMD", test vectors
RIPEMD_VECTORS = [
    (b"", "9c1185a5c5e9fc54612808977ee8f548b2258d31"),
    (b"a", "0bdc9d2d256b3ee9daae347be6f4dc835a467ffe"),
    (b"abc", "8eb208f7e05d987a9b044a8e98c6b087f15a0bfc"),
    (b"message digest", "5d0689ef49d2fae572b881b123a85ffa21595f36"),
    (b"abcdefghijklmnopqrstuvwxyz", "f71c27109c692c1b56bbdceb5b9d2865b3708dbc"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "12a053384a9c0c88e405a06c27dcf49ada62eb2b"),
    (b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
     "b0e20b6e3116640286ed3a87a5713079b21f5189"),
    (b"1234567890" * 8, "9b752e45573d4b39f4dbd3323cab82bf63326bfb"),
]


@pytest.fixture(scope="module")
def so():
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in DEPS):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO] + SRC)
    return SO


def _check(so_path):
    L = ctypes.CDLL(so_path)
    rng = random.Random(11)
    out = ctypes.create_string_buffer(32)
    for n in list(range(0, 200)) + [255, 256, 257, 1000, 4096, 10007]:
        m = bytes(rng.getrandbits(8) for _ in range(n))
        L.th_sha256(m, n, out)
        assert out.raw == hashlib.sha256(m).digest(), n
        L.th_sha1(m, n, out)
        assert out.raw[:20] == hashlib.sha1(m).digest(), n
    for m, h in RIPEMD_VECTORS:
        L.th_ripemd160(m, len(m), out)
        assert out.raw[:20].hex() == h, m
    try:
        hashlib.new("ripemd160")
    except ValueError:
        return L.th_shani()
    for n in (0, 1, 33, 55, 56, 63, 64, 65, 119, 120, 128, 500):
        m = bytes(rng.getrandbits(8) for _ in range(n))
        L.th_ripemd160(m, n, out)
        assert out.raw[:20] == hashlib.new("ripemd160", m).digest(), n
        L.th_hash160(m, n, out)
        assert out.raw[:20] == hashlib.new("ripemd160", hashlib.sha256(m).digest()).digest(), n
    return L.th_shani()


def test_host_hashes_default_path(so):
    _check(so)


def test_host_sha256_portable_path(so):
    """The portable SHA-256 compression (forced with BCC_NO_SHANI) in a fresh process."""
    code = f"import sys; sys.path.insert(0, {HERE!r}); import test_host_hashes as t; print(t._check({so!r}))"
    env = dict(os.environ, BCC_NO_SHANI="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == "0"


def test_host_hash160_batch_other_paths(so):
    """The same check with AVX-512 off (eight RIPEMD-160s per AVX2 pass) and with both off."""
    for env in ({"BCC_NO_AVX512": "1"}, {"BCC_NO_AVX512": "1", "BCC_NO_AVX2": "1"}):
        code = ("import sys; sys.path.insert(0, %r); import test_host_hashes as T; "
                "T.test_host_hash160_batch_matches_scalar(%r); print('ok')" % (os.path.dirname(__file__), so))
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, **env),
                           capture_output=True, text=True)
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (env, r.stderr[-2000:])


def test_host_hash160_batch_matches_scalar(so):
    """hash160_batch (sixteen SHA-256s and RIPEMD-160s per AVX-512 pass, eight RIPEMD-160s per AVX2
    pass, the scalar path for the rest) against hash160 on the same messages: key-sized and
    odd-sized inputs, batch sizes that leave remainders."""
    import ctypes
    import random
    L = ctypes.CDLL(so)
    rng = random.Random(160)
    cases = [(count, [33, 65, 0, 1, 31, 32, 55, 56, 64, 100, 200]) for count in (1, 7, 8, 9, 16, 23, 64)]
    cases += [(count, [33, 0, 1, 20, 32, 54, 55]) for count in (16, 17, 33, 64)]  # one-block SHA-256s
    cases += [(64, [33])]
    for count, sizes in cases:
        msgs = [rng.randbytes(rng.choice(sizes)) for _ in range(count)]
        n = (ctypes.c_ulong * count)(*[len(m) for m in msgs])
        out = ctypes.create_string_buffer(20 * count)
        L.th_hash160_batch(b"".join(msgs), n, ctypes.c_ulong(count), out)
        for i, m in enumerate(msgs):
            exp = ctypes.create_string_buffer(20)
            L.th_hash160(m, len(m), exp)
            assert out.raw[20 * i: 20 * i + 20] == exp.raw, (count, i, len(m))


def test_device_key_hash160(so):
    """The device-side key HASH160 (sha256_device.h key_hash160: SHA-256 of the 33- / 65-byte key
    built from a tuple row, then RIPEMD-160, the P2WPKH / P2PKH EQUALVERIFY check deferred to the
    GPU) compiled as host code, against the host HASH160 of the same key bytes."""
    L = ctypes.CDLL(so)
    rng = random.Random(23)
    out = ctypes.create_string_buffer(20)
    ref = ctypes.create_string_buffer(32)
    for i in range(400):
        tag = (2, 3, 4, 6, 7)[i % 5]
        x = bytes(rng.getrandbits(8) for _ in range(32))
        y = bytes(rng.getrandbits(8) for _ in range(32))
        key = bytes([tag]) + x + (y if tag >= 4 else b"")
        L.th_key_hash160(tag, x, y, out)
        L.th_hash160(key, len(key), ref)
        assert out.raw == ref.raw[:20], (tag, i)
