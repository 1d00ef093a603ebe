"""The engine's HOST code with the device pipeline replaced by the oracle (test-only build:
tests/native/engine_host_stub.cpp + csrc/host/*.cpp + oracle/bcc_oracle.c ->
tests/native/_build/engine_host.so).  Lets the CPU suite run the product's host logic (parser,
interpreter, deferring checker, job builder, round stitching, device sharding, failure handling)
without a GPU; the -m gpu tests run the same paths through librbc_amd.so."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SO = os.path.join(HERE, "native", "_build", "engine_host.so")


def load():
    srcs = [os.path.join(HERE, "native", "engine_host_stub.cpp")]
    hostdir = os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc", "host")
    srcs += [os.path.join(hostdir, f) for f in sorted(os.listdir(hostdir)) if f.endswith(".cpp")]
    deps = srcs + [os.path.join(hostdir, f) for f in os.listdir(hostdir) if f.endswith(".h")]
    csrc = os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc")
    deps += [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith(".h")]  # lane code
    deps += [os.path.join(ROOT, "oracle", "bcc_oracle.c"),
             os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc", "pipeline.h"),
             os.path.join(ROOT, "include", "bcc_amd.h"),
             os.path.join(ROOT, "include", "bitcoinconsensus.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        tmp = SO + f".{os.getpid()}.tmp"
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread",
                               "-I" + os.path.join(ROOT, "include"),
                               "-I" + os.path.join(ROOT, "rust-bitcoinconsensus_amd", "csrc"),
                               "-o", tmp] + srcs + ["-x", "c", os.path.join(ROOT, "oracle", "bcc_oracle.c")])
        os.replace(tmp, SO)
    L = ctypes.CDLL(SO)
    L.bitcoinconsensus_verify_batch.restype = ctypes.c_long
    L.bcc_debug_fail_device_rounds.argtypes = [ctypes.c_int]
    L.bcc_set_device_failure_policy.argtypes = [ctypes.c_int]
    L.bcc_get_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.bcc_set_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.bcc_pubkey_verify_batch.argtypes = [ctypes.c_char_p, u64p, ctypes.c_char_p, ctypes.c_char_p,
                                          u64p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
    import bitcoinconsensus_amd as B
    L.bcc_taproot_verify_batch.argtypes = [ctypes.POINTER(B.TaprootCheck), ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_int), ctypes.c_void_p,
                                           ctypes.c_int]
    return L


def set_devices(L, devs):
    arr = (ctypes.c_int * max(1, len(devs)))(*devs)
    assert L.bcc_set_devices(arr, len(devs)) == 0


def tuple_blobs(ts):
    """(pub_blob, pub_off, msg, sig_blob, sig_off) ctypes args for bcc_pubkey_verify_batch."""
    def blob(parts):
        off = [0]
        for p in parts:
            off.append(off[-1] + len(p))
        return b"".join(parts), (ctypes.c_uint64 * len(off))(*off)
    pb, po = blob([t["pub"] for t in ts])
    sb, so = blob([t["sig"] for t in ts])
    return pb, po, b"".join(t["hash"] for t in ts), sb, so


def pubkey_verify(L, ts, device=0):
    pb, po, msg, sb, so = tuple_blobs(ts)
    out = ctypes.create_string_buffer(max(1, len(ts)))
    assert L.bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, len(ts), device) == 0
    return out.raw[: len(ts)]
