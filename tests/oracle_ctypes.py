"""ctypes access to the CHECKERS (test infrastructure only).

* ``Oracle``    — the plain-C restatement, oracle/_build/libbcc_oracle.so (oracle/bcc_oracle.c)
* ``Reference`` — the reference itself, oracle/_ref/libref_consensus.so, compiled from
                  /root/reference by oracle/Makefile (present here and shipped to the GPU box).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libbcc_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_consensus.so")

c_u8p = ctypes.c_char_p
c_sz = ctypes.c_size_t


def _build_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])


class Oracle:
    """CPU restatement of the hot path (oracle/bcc_oracle.h)."""

    def __init__(self):
        _build_oracle()
        L = ctypes.CDLL(ORACLE_SO)
        self.L = L
        L.bcco_sha256.argtypes = [c_u8p, c_sz, c_u8p]
        L.bcco_sha256d.argtypes = [c_u8p, c_sz, c_u8p]
        L.bcco_der_parse_lax.argtypes = [c_u8p, c_sz, c_u8p, c_u8p]
        L.bcco_pubkey_parse.argtypes = [c_u8p, c_sz, c_u8p, c_u8p]
        L.bcco_ecdsa_verify_raw.argtypes = [c_u8p] * 5
        L.bcco_pubkey_verify.argtypes = [c_u8p, c_sz, c_u8p, c_u8p, c_sz]
        L.bcco_schnorr_verify.argtypes = [c_u8p, c_u8p, c_u8p]
        L.bcco_ecmult_gen.argtypes = [c_u8p, c_u8p, c_u8p]
        L.bcco_sighash.argtypes = [c_u8p, c_sz, ctypes.c_uint, c_u8p, c_sz, ctypes.c_int,
                                   ctypes.c_int64, ctypes.c_int, c_u8p]
        L.bcco_sighash_schnorr.argtypes = [c_u8p, c_sz, c_u8p, c_sz, ctypes.c_uint, ctypes.c_int,
                                           ctypes.c_int, c_u8p, c_sz, c_u8p, ctypes.c_uint32,
                                           c_u8p]
        L.bcco_taproot_check.argtypes = [c_u8p, c_sz, c_u8p, c_sz, ctypes.c_uint, c_u8p, c_sz,
                                         c_u8p, ctypes.c_int, c_u8p, c_sz, c_u8p, ctypes.c_uint32,
                                         ctypes.POINTER(ctypes.c_int), c_u8p]

    def sha256(self, b):
        o = ctypes.create_string_buffer(32)
        self.L.bcco_sha256(b, len(b), o)
        return o.raw

    def sha256d(self, b):
        o = ctypes.create_string_buffer(32)
        self.L.bcco_sha256d(b, len(b), o)
        return o.raw

    def der_parse_lax(self, sig):
        r = ctypes.create_string_buffer(32)
        s = ctypes.create_string_buffer(32)
        ok = self.L.bcco_der_parse_lax(sig, len(sig), r, s)
        return ok, r.raw, s.raw

    def pubkey_parse(self, pub):
        x = ctypes.create_string_buffer(32)
        y = ctypes.create_string_buffer(32)
        ok = self.L.bcco_pubkey_parse(pub, len(pub), x, y)
        return (x.raw, y.raw) if ok else None

    def ecdsa_verify_raw(self, qx, qy, r, s, msg):
        return self.L.bcco_ecdsa_verify_raw(qx, qy, r, s, msg)

    def pubkey_verify(self, pub, hash32, sig):
        return self.L.bcco_pubkey_verify(pub, len(pub), hash32, sig, len(sig))

    def schnorr_verify(self, sig64, msg32, xonly32):
        return self.L.bcco_schnorr_verify(sig64, msg32, xonly32)

    def ecmult_gen(self, k32):
        x = ctypes.create_string_buffer(32)
        y = ctypes.create_string_buffer(32)
        ok = self.L.bcco_ecmult_gen(k32, x, y)
        return (x.raw, y.raw) if ok else None

    def sighash(self, tx, nin, script, hashtype, amount, sigversion):
        o = ctypes.create_string_buffer(32)
        ok = self.L.bcco_sighash(tx, len(tx), nin, script, len(script), hashtype, amount,
                                 sigversion, o)
        return o.raw if ok else None

    def sighash_schnorr(self, tx, spent, nin, hash_type, sigversion, annex=None,
                        tapleaf=bytes(32), codesep=0xFFFFFFFF):
        """(rc, sighash): rc 1 ok, 0 reference returns false, -1 refused inputs."""
        o = ctypes.create_string_buffer(32)
        rc = self.L.bcco_sighash_schnorr(tx, len(tx), spent, len(spent), nin, hash_type,
                                         sigversion, annex, len(annex or b""), tapleaf, codesep, o)
        return rc, o.raw

    def taproot_check(self, tx, spent, nin, sig, pk, sigversion, annex=None, tapleaf=bytes(32),
                      codesep=0xFFFFFFFF):
        """(ret, serror) of CheckSchnorrSignature; ret -1 for refused inputs."""
        e = ctypes.c_int(0)
        h = ctypes.create_string_buffer(32)
        r = self.L.bcco_taproot_check(tx, len(tx), spent, len(spent), nin, sig, len(sig), pk,
                                      sigversion, annex, len(annex or b""), tapleaf, codesep,
                                      ctypes.byref(e), h)
        return r, e.value


class Reference:
    """The reference (Bitcoin Core v0.21 libbitcoinconsensus + libsecp256k1), see ref_shim.cpp."""

    def __init__(self):
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(REF_SO)
        L = ctypes.CDLL(REF_SO)
        self.L = L
        L.ref_verify_script_with_amount.argtypes = [c_u8p, ctypes.c_uint, ctypes.c_int64, c_u8p,
                                                    ctypes.c_uint, ctypes.c_uint, ctypes.c_uint,
                                                    ctypes.POINTER(ctypes.c_int)]
        L.ref_verify_script.argtypes = [c_u8p, ctypes.c_uint, c_u8p, ctypes.c_uint, ctypes.c_uint,
                                        ctypes.c_uint, ctypes.POINTER(ctypes.c_int)]
        L.ref_pubkey_verify.argtypes = [c_u8p, c_sz, c_u8p, c_u8p, c_sz]
        L.ref_schnorr_verify.argtypes = [c_u8p, c_u8p, c_u8p]
        L.ref_pubkey_create.argtypes = [c_u8p, ctypes.c_int, c_u8p, ctypes.POINTER(c_sz)]
        L.ref_sign.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.POINTER(c_sz)]
        L.ref_schnorr_sign.argtypes = [c_u8p, c_u8p, c_u8p, c_u8p, c_u8p]
        i32p = ctypes.POINTER(ctypes.c_int)
        L.ref_capture_script.argtypes = [c_u8p, ctypes.c_uint, ctypes.c_int64, c_u8p, ctypes.c_uint,
                                         ctypes.c_uint, ctypes.c_uint, ctypes.c_int, c_u8p, i32p,
                                         c_u8p, i32p, c_u8p, i32p, i32p, i32p]
        L.ref_bench_verify_script.restype = ctypes.c_double
        L.ref_bench_pubkey_verify.restype = ctypes.c_double
        vp = ctypes.c_void_p
        L.ref_bench_pubkey_verify_blob.argtypes = [ctypes.c_int, ctypes.c_long] + [vp] * 6
        L.ref_bench_pubkey_verify_blob.restype = ctypes.c_double
        L.ref_bench_schnorr_verify.argtypes = [ctypes.c_int, ctypes.c_long] + [vp] * 4
        L.ref_bench_schnorr_verify.restype = ctypes.c_double
        L.ref_bulk_verify_script.argtypes = [ctypes.c_int, ctypes.c_long] + [vp] * 6 + [
            ctypes.c_uint, vp, vp]
        L.ref_bulk_verify_script.restype = ctypes.c_double
        L.ref_taproot_check.argtypes = [c_u8p, c_sz, c_u8p, c_sz, ctypes.c_uint, c_u8p, c_sz,
                                        c_u8p, ctypes.c_int, c_u8p, c_sz, c_u8p, ctypes.c_uint32,
                                        i32p, c_u8p, i32p]

    def verify_script_with_amount(self, spk, amount, tx, nin, flags):
        e = ctypes.c_int(0)
        r = self.L.ref_verify_script_with_amount(spk, len(spk), amount, tx, len(tx), nin, flags,
                                                 ctypes.byref(e))
        return r, e.value

    def verify_script(self, spk, tx, nin, flags):
        e = ctypes.c_int(0)
        r = self.L.ref_verify_script(spk, len(spk), tx, len(tx), nin, flags, ctypes.byref(e))
        return r, e.value

    def pubkey_verify(self, pub, hash32, sig):
        return self.L.ref_pubkey_verify(pub, len(pub), hash32, sig, len(sig))

    def schnorr_verify(self, sig64, msg32, xonly32):
        return self.L.ref_schnorr_verify(sig64, msg32, xonly32)

    def bulk_verify_script(self, items, flags, threads=None):
        """bitcoinconsensus_verify_script_with_amount over (spk, amount, tx, nin) items on a
        dynamically chunked thread pool.  Returns ([(ret, err)], wall seconds)."""
        import numpy as np
        items = list(items)
        n = len(items)
        if threads is None:
            threads = max(1, min(16, len(os.sched_getaffinity(0))))

        def blob(parts):
            off = np.zeros(len(parts) + 1, np.int64)
            off[1:] = np.cumsum([len(p) for p in parts])
            return np.frombuffer(b"".join(parts) + b"\0", np.uint8), off

        sb, so = blob([bytes(it[0]) for it in items])
        tb, to = blob([bytes(it[2]) for it in items])
        am = np.array([it[1] - (1 << 64) if it[1] >= (1 << 63) else it[1] for it in items],
                      np.int64)
        nin = np.array([it[3] & 0xffffffff for it in items], np.uint32)
        ret = np.zeros(max(n, 1), np.int32)
        err = np.zeros(max(n, 1), np.int32)
        p = lambda a: a.ctypes.data  # noqa: E731
        secs = self.L.ref_bulk_verify_script(threads, n, p(sb), p(so), p(tb), p(to), p(am), p(nin),
                                             flags & 0xffffffff, p(ret), p(err))
        return [(int(ret[i]), int(err[i])) for i in range(n)], secs

    def pubkey_verify_blob(self, pub_blob, pub_off, msg32, sig_blob, sig_off, threads=1, n=None):
        """CPubKey::Verify over numpy blob inputs (uint64 offsets) on `threads` host threads.
        Returns (verdicts as a uint8 numpy array, wall seconds)."""
        import numpy as np
        n = len(pub_off) - 1 if n is None else n
        out = np.zeros(max(n, 1), np.uint8)
        p = lambda a: a.ctypes.data  # noqa: E731
        t = self.L.ref_bench_pubkey_verify_blob(threads, n, p(pub_blob), p(pub_off), p(msg32),
                                                p(sig_blob), p(sig_off), p(out))
        return out[:n], t

    def schnorr_verify_rows(self, sig64, msg32, xonly32, threads=1, n=None):
        """secp256k1_schnorrsig_verify over numpy row arrays.  Returns (verdicts, seconds)."""
        import numpy as np
        n = len(msg32) // 32 if n is None else n
        out = np.zeros(max(n, 1), np.uint8)
        p = lambda a: a.ctypes.data  # noqa: E731
        t = self.L.ref_bench_schnorr_verify(threads, n, p(sig64), p(msg32), p(xonly32), p(out))
        return out[:n], t

    def taproot_check(self, tx, spent, nin, sig, pk, sigversion, annex=None, tapleaf=bytes(32),
                      codesep=0xFFFFFFFF):
        """CheckSchnorrSignature (interpreter.cpp:1678-1704) -> (ret, serror, sighash or None);
        ret -1 where the reference would assert (unparsable tx / spent outputs, counts)."""
        e = ctypes.c_int(0)
        hashed = ctypes.c_int(0)
        h = ctypes.create_string_buffer(32)
        r = self.L.ref_taproot_check(tx, len(tx), spent, len(spent), nin, sig, len(sig), pk,
                                     sigversion, annex, len(annex or b""), tapleaf, codesep,
                                     ctypes.byref(e), h, ctypes.byref(hashed))
        return r, e.value, (h.raw if hashed.value else None)

    def pubkey_create(self, sk, compressed=True):
        out = ctypes.create_string_buffer(65)
        n = c_sz(65)
        if not self.L.ref_pubkey_create(sk, 1 if compressed else 0, out, ctypes.byref(n)):
            return None
        return out.raw[: n.value]

    def sign(self, sk, msg32):
        out = ctypes.create_string_buffer(72)
        n = c_sz(72)
        if not self.L.ref_sign(sk, msg32, out, ctypes.byref(n)):
            return None
        return out.raw[: n.value]

    def schnorr_sign(self, sk, msg32, aux32):
        sig = ctypes.create_string_buffer(64)
        xo = ctypes.create_string_buffer(32)
        if not self.L.ref_schnorr_sign(sk, msg32, aux32, sig, xo):
            return None
        return sig.raw, xo.raw

    def capture_script(self, spk, amount, tx, nin, flags, cap=64):
        pub = ctypes.create_string_buffer(65 * cap)
        sig = ctypes.create_string_buffer(80 * cap)
        h = ctypes.create_string_buffer(32 * cap)
        publen = (ctypes.c_int * cap)()
        siglen = (ctypes.c_int * cap)()
        verdict = (ctypes.c_int * cap)()
        ncap = ctypes.c_int(0)
        serr = ctypes.c_int(0)
        r = self.L.ref_capture_script(spk, len(spk), amount, tx, len(tx), nin, flags, cap, pub,
                                      publen, sig, siglen, h, verdict, ctypes.byref(ncap),
                                      ctypes.byref(serr))
        recs = []
        for i in range(min(cap, ncap.value)):
            recs.append(dict(pub=pub.raw[65 * i: 65 * i + publen[i]],
                             sig=sig.raw[80 * i: 80 * i + min(80, siglen[i])],
                             sighash=h.raw[32 * i: 32 * i + 32], verdict=verdict[i]))
        return r, serr.value, recs


def reference_available():
    return os.path.exists(REF_SO)
