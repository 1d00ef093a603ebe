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
BENCH_LIB_PATH = os.path.join(_HERE, "librbc_bench.so")

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


# Engine-specific code (include/bitcoinconsensus.h BCC_ERR_DEVICE_FAILURE), outside the mirrored
# enum: only verify_batch_raw can report it, for items the device left without a verdict.
ERR_DEVICE_FAILURE = 6


class DeviceFailure(enum.IntEnum):
    """The one code a batch item can carry beyond the crate's Error: 'no verdict' (the device
    round that item needed failed under DEVICE_FAILURE_ERROR).  Never a consensus result."""
    ERR_DEVICE_FAILURE = ERR_DEVICE_FAILURE


def error_from_code(code):
    """An err_out code of the batch ABI -> Error (0-5, lib.rs:172-185) or
    DeviceFailure.ERR_DEVICE_FAILURE (6).  Anything else is a ValueError: the crate's repr(C)
    enum has no other discriminant, so an unknown code must never be cast to it."""
    code = int(code)
    if 0 <= code <= 5:
        return Error(code)
    if code == ERR_DEVICE_FAILURE:
        return DeviceFailure.ERR_DEVICE_FAILURE
    raise ValueError(f"unknown bitcoinconsensus error code {code}")


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
        L.mi_schnorr_verify_tuples.argtypes = [u8p, u8p, u8p, u8p, sz, ctypes.c_int]
        L.mi_schnorr_verify_device.argtypes = [vp] * 4 + [sz, vp]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.bcc_pubkey_verify_batch.argtypes = [u8p, u64p, u8p, u8p, u64p, u8p, sz, ctypes.c_int]
        L.bcc_taproot_verify_batch.argtypes = [ctypes.POINTER(TaprootCheck), sz,
                                               ctypes.POINTER(ctypes.c_int),
                                               ctypes.POINTER(ctypes.c_int), vp, ctypes.c_int]
        L.bcc_debug_scratch_cap_lanes.argtypes = [sz]
        _bind_consensus(L)
        L.bcc_source_hash.restype = ctypes.c_char_p
        _lib = L
    return _lib


_blib = None


def blib():
    """Load librbc_bench.so (synthetic workloads, generators, microbenchmark: include/bcc_bench.h),
    which links the product library; raises if it has not been built."""
    global _blib
    if _blib is None:
        lib()
        if not os.path.exists(BENCH_LIB_PATH):
            raise ImportError(f"{BENCH_LIB_PATH} missing: build with `make -C {_HERE}`")
        L = ctypes.CDLL(BENCH_LIB_PATH)
        u8p, sz, vp, ui = ctypes.c_char_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_uint
        L.mi_microbench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        dp = ctypes.POINTER(ctypes.c_double)
        L.mi_primbench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp]
        L.mi_microbench_sustained.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                              ctypes.c_double, ctypes.c_int, dp, dp, dp]
        L.bcc_tupleset_c4.argtypes = [sz, ctypes.c_uint64, ctypes.c_int]
        L.bcc_tupleset_c4.restype = vp
        L.bcc_tupleset_c4_range.argtypes = [sz, ctypes.c_uint64, sz, sz, ctypes.c_int]
        L.bcc_tupleset_c4_range.restype = vp
        L.bcc_tupleset_c5.argtypes = [sz, ctypes.c_uint64, u8p, u8p, u8p, u8p, sz, ctypes.c_int]
        L.bcc_tupleset_c5.restype = vp
        L.bcc_tupleset_c5_range.argtypes = [sz, ctypes.c_uint64, sz, u8p, u8p, u8p, u8p, sz,
                                            ctypes.c_int]
        L.bcc_tupleset_c5_range.restype = vp
        L.bcc_tupleset_free.argtypes = [vp]
        L.bcc_tupleset_size.argtypes = [vp]
        L.bcc_tupleset_size.restype = sz
        L.bcc_tupleset_run.argtypes = [vp, vp]
        L.bcc_tupleset_verdicts.argtypes = [vp, u8p]
        L.bcc_tupleset_view.argtypes = [vp, ctypes.POINTER(TuplesetHost)]
        L.bcc_workload_p2wpkh.argtypes = [sz, ctypes.c_uint64, ctypes.c_int]
        L.bcc_workload_p2wpkh.restype = vp
        L.bcc_workload_p2wpkh_range.argtypes = [sz, ctypes.c_uint64, sz, ctypes.c_int]
        L.bcc_workload_p2wpkh_range.restype = vp
        u32p = ctypes.POINTER(ctypes.c_uint32)
        L.bcc_workload_block.argtypes = [u32p, u32p, sz, ctypes.c_uint64, ctypes.c_int]
        L.bcc_workload_block.restype = vp
        L.bcc_workload_items.argtypes = [vp, ctypes.POINTER(sz)]
        L.bcc_workload_items.restype = ctypes.POINTER(BatchItem)
        L.bcc_workload_free.argtypes = [vp]
        L.bcc_workload_size.argtypes = [vp]
        L.bcc_workload_size.restype = sz
        for f in (L.bcc_workload_run, L.bcc_workload_run_sighash, L.bcc_workload_run_ecdsa):
            f.argtypes = [vp, vp]
        L.bcc_workload_verdicts.argtypes = [vp, u8p, sz]
        L.bcc_workload_from_items.argtypes = [ctypes.POINTER(BatchItem), sz, ui, ctypes.c_int]
        L.bcc_workload_from_items.restype = vp
        L.bcc_workload_tuple_items.argtypes = [vp, ctypes.POINTER(ctypes.c_uint32), sz]
        L.bcc_workload_msgs.argtypes = [vp, u8p, sz]
        szp = ctypes.POINTER(sz)
        L.bcc_workload_shape.argtypes = [vp, szp, szp, szp, szp, szp]
        L.bcc_workload_sighash_bytes.argtypes = [vp]
        L.bcc_workload_sighash_bytes.restype = sz
        L.bcc_workload_item.argtypes = [vp, sz, u8p, szp, ctypes.POINTER(ctypes.c_int64), u8p, sz]
        L.bcc_workload_item.restype = sz
        L.bcc_debug_sighash.argtypes = [ctypes.POINTER(SighashCheck), sz, u8p, ctypes.c_int]
        L.mi_gen_pubkeys.argtypes = [u8p, sz, u8p, u8p, u8p, ctypes.c_int]
        L.mi_gen_sign.argtypes = [u8p, u8p, u8p, sz, u8p, u8p, u8p, ctypes.c_int]
        L.mi_gen_schnorr_sign.argtypes = [u8p, u8p, u8p, sz, u8p, u8p, u8p, ctypes.c_int]

        _blib = L
    return _blib


def source_hash():
    """Hash of the sources the loaded library was built from (Makefile / source_hash.py)."""
    return lib().bcc_source_hash().decode()


class BatchItem(ctypes.Structure):
    """struct bcc_batch_item (include/bitcoinconsensus.h)."""
    _fields_ = [("script_pubkey", ctypes.c_void_p), ("script_pubkey_len", ctypes.c_uint),
                ("amount", ctypes.c_int64), ("tx_to", ctypes.c_void_p),
                ("tx_to_len", ctypes.c_uint), ("n_in", ctypes.c_uint)]


class SighashCheck(ctypes.Structure):
    """struct bcc_sighash_check (include/bcc_bench.h)."""
    _fields_ = [("tx", ctypes.c_void_p), ("tx_len", ctypes.c_size_t),
                ("script_code", ctypes.c_void_p), ("script_code_len", ctypes.c_size_t),
                ("n_in", ctypes.c_uint), ("hashtype", ctypes.c_int32), ("amount", ctypes.c_int64),
                ("sigversion", ctypes.c_int)]


def debug_sighash(checks, device=0):
    """The GPU sighash stage alone (bcc_debug_sighash): checks = [(tx, script_code, n_in,
    hashtype, amount, sigversion)], each built into a device job exactly as the batch engine's
    deferring checker builds it.  Returns the n 32-byte message rows (raw uint256 bytes)."""
    n = len(checks)
    if n == 0:
        return []
    arr = (SighashCheck * n)()
    keep = []
    for i, (tx, code, nin, ht, amount, sv) in enumerate(checks):
        tb, cb = ctypes.create_string_buffer(bytes(tx), max(1, len(tx))), \
            ctypes.create_string_buffer(bytes(code), max(1, len(code)))
        keep += [tb, cb]
        ht = int(ht) & 0xffffffff
        arr[i] = SighashCheck(ctypes.addressof(tb), len(tx), ctypes.addressof(cb), len(code), nin,
                              ht - (1 << 32) if ht >= 1 << 31 else ht, amount, sv)
    out = ctypes.create_string_buffer(32 * n)
    rc = blib().bcc_debug_sighash(arr, n, out, device)
    if rc != 0:
        raise RuntimeError(f"bcc_debug_sighash failed: {rc}")
    return [out.raw[32 * i:32 * i + 32] for i in range(n)]


class TuplesetHost(ctypes.Structure):
    """struct bcc_tupleset_host (include/bcc_amd.h)."""
    _fields_ = [("n", ctypes.c_size_t)] + [
        (f, ctypes.c_void_p) for f in ("pub_blob", "sig_blob", "msg32", "sig64", "xonly32", "cls",
                                       "expect", "pub_off", "sig_off")]


class BatchStats(ctypes.Structure):
    _fields_ = [("items", ctypes.c_size_t), ("tuples", ctypes.c_size_t),
                ("rounds", ctypes.c_size_t), ("preimages", ctypes.c_size_t),
                ("aux_messages", ctypes.c_size_t), ("host_rejected", ctypes.c_size_t),
                ("host_seconds", ctypes.c_double), ("gpu_seconds", ctypes.c_double),
                ("prepare_seconds", ctypes.c_double), ("interpret_seconds", ctypes.c_double),
                ("merge_seconds", ctypes.c_double), ("stage_seconds", ctypes.c_double),
                ("total_seconds", ctypes.c_double), ("device_retries", ctypes.c_size_t),
                ("devices", ctypes.c_size_t), ("host_rounds", ctypes.c_size_t),
                ("host_hashed", ctypes.c_size_t), ("shard_seconds", ctypes.c_double),
                ("stitch_seconds", ctypes.c_double), ("finish_seconds", ctypes.c_double),
                ("host_jobs_seconds", ctypes.c_double), ("prepare_lag_seconds", ctypes.c_double),
                ("prepare_parse_seconds", ctypes.c_double), ("prepare_hash_seconds", ctypes.c_double),
                ("device_key_hashes", ctypes.c_size_t),
                ("interpret_shard_max_seconds", ctypes.c_double),
                ("interpret_shard_mean_seconds", ctypes.c_double),
                ("process_cpu_seconds", ctypes.c_double),
                ("process_cpu_in_gpu_wait_seconds", ctypes.c_double),
                ("early_rows", ctypes.c_size_t), ("early_mapped", ctypes.c_size_t),
                ("early_seconds", ctypes.c_double), ("early_msgs", ctypes.c_size_t)]


def _bind_consensus(L):
    u8p, ui = ctypes.c_char_p, ctypes.c_uint
    ip = ctypes.POINTER(ctypes.c_int)
    L.bitcoinconsensus_verify_script_with_amount.argtypes = [u8p, ui, ctypes.c_int64, u8p, ui, ui,
                                                             ui, ip]
    L.bitcoinconsensus_verify_script.argtypes = [u8p, ui, u8p, ui, ui, ui, ip]
    L.bitcoinconsensus_version.restype = ui
    L.bitcoinconsensus_verify_batch.argtypes = [ctypes.POINTER(BatchItem), ctypes.c_size_t, ui,
                                                ip, ip]
    L.bitcoinconsensus_verify_batch.restype = ctypes.c_long
    L.bcc_set_device.argtypes = [ctypes.c_int]
    L.bcc_debug_fail_device_rounds.argtypes = [ctypes.c_int]
    L.bcc_set_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.bcc_get_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.bcc_last_batch_stats.argtypes = [ctypes.POINTER(BatchStats)]
    L.bcc_set_device_failure_policy.argtypes = [ctypes.c_int]
    L.bcc_set_host_small_round.argtypes = [ctypes.c_size_t]
    L.bcc_host_fallback_rounds.restype = ctypes.c_size_t
    L.bcc_debug_fail_device_rounds_code.argtypes = [ctypes.c_int, ctypes.c_int]
    L.bcc_host_verify_tuples.argtypes = [ctypes.c_char_p] * 5 + [ctypes.c_size_t, ctypes.c_uint]


class Workload:
    """A synthetic workload staged in HBM (include/bcc_amd.h, bcc_workload_*).

    kind "p2wpkh": config C2, n one-input P2WPKH spends.
    kind "block":  config C3, transactions shaped by `shape` = [(n_inputs, n_outputs), ...]
                   (one item per input)."""

    def __init__(self, n=0, seed=0x5EED0001, device=0, kind="p2wpkh", shape=None, items=None,
                 flags=VERIFY_ALL, first=0):
        if kind == "items":  # any caller items, staged through the same first-round pass
            arr, keep = _batch_items(items)
            self.h = blib().bcc_workload_from_items(arr, len(keep[0]), flags & 0xffffffff, device)
        elif kind == "p2wpkh":  # spends [first, first + n) of the global set from `seed`
            self.h = blib().bcc_workload_p2wpkh_range(n, seed, first, device)
        elif kind == "block":
            nin = (ctypes.c_uint32 * len(shape))(*[a for a, _ in shape])
            nout = (ctypes.c_uint32 * len(shape))(*[b for _, b in shape])
            self.h = blib().bcc_workload_block(nin, nout, len(shape), seed, device)
        else:
            raise ValueError(kind)
        if not self.h:
            raise RuntimeError(f"bcc_workload_{kind} failed")
        self.n = blib().bcc_workload_size(self.h)
        self.kind = kind

    def verify_batch(self, flags=VERIFY_ALL):
        """bitcoinconsensus_verify_batch over all items (host interpreter + GPU rounds, end to
        end, host buffers as the drop-in receives them).  Returns (n_valid, ret bytes)."""
        cnt = ctypes.c_size_t(0)
        items = blib().bcc_workload_items(self.h, ctypes.byref(cnt))
        ret = (ctypes.c_int * max(1, cnt.value))()
        rc = lib().bitcoinconsensus_verify_batch(items, cnt.value, flags & 0xffffffff, ret, None)
        if rc < 0:
            raise RuntimeError("bitcoinconsensus_verify_batch: device pipeline failed")
        return rc, bytes(memoryview(ret).cast("B"))[:: ctypes.sizeof(ctypes.c_int)][: cnt.value]

    def run(self, stream=None):
        rc = blib().bcc_workload_run(self.h, stream)
        if rc:
            raise RuntimeError(f"bcc_workload_run: {rc}")

    def run_sighash(self, stream=None):
        rc = blib().bcc_workload_run_sighash(self.h, stream)
        if rc:
            raise RuntimeError(f"bcc_workload_run_sighash: {rc}")

    def run_ecdsa(self, stream=None):
        rc = blib().bcc_workload_run_ecdsa(self.h, stream)
        if rc:
            raise RuntimeError(f"bcc_workload_run_ecdsa: {rc}")

    def verdicts(self):
        """One byte per staged tuple row (a block workload's multisig inputs have several rows:
        the buffer is sized by rows, not items)."""
        t = self.shape()["tuples"]
        out = ctypes.create_string_buffer(max(1, t))
        rc = blib().bcc_workload_verdicts(self.h, out, len(out))
        if rc:
            raise RuntimeError(f"bcc_workload_verdicts: {rc}")
        return out.raw[:t]

    def tuple_items(self):
        """Item index of every staged tuple row."""
        t = self.shape()["tuples"]
        out = (ctypes.c_uint32 * max(1, t))()
        if blib().bcc_workload_tuple_items(self.h, out, len(out)):
            raise RuntimeError("bcc_workload_tuple_items failed")
        return list(out)[:t]

    def msgs(self):
        """The sighash rows (32 bytes per staged tuple) of the last run."""
        t = self.shape()["tuples"]
        out = ctypes.create_string_buffer(max(1, 32 * t))
        if blib().bcc_workload_msgs(self.h, out, len(out)):
            raise RuntimeError("bcc_workload_msgs failed")
        return out.raw[: 32 * t]

    def shape(self):
        v = [ctypes.c_size_t() for _ in range(5)]
        blib().bcc_workload_shape(self.h, *[ctypes.byref(x) for x in v])
        d = dict(zip(("tuples", "sighash_blocks", "aux_blocks", "preimages", "aux_messages"),
                     (x.value for x in v)))
        d["sighash_bytes"] = blib().bcc_workload_sighash_bytes(self.h)
        return d

    def item(self, i):
        """(spent script, amount, tx bytes, input index) of item i."""
        cnt = ctypes.c_size_t(0)
        it = blib().bcc_workload_items(self.h, ctypes.byref(cnt))[i]
        return (ctypes.string_at(it.script_pubkey, it.script_pubkey_len), it.amount,
                ctypes.string_at(it.tx_to, it.tx_to_len), it.n_in)

    def free(self):
        if self.h:
            blib().bcc_workload_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def version():
    """Returns libbitcoinconsensus API version (src/lib.rs:68)."""
    return lib().bitcoinconsensus_version()


def verify_script_with_amount(spk, amount, tx, n_in, flags):
    """Raw C-ABI call: returns (ret, err) exactly as bitcoinconsensus_verify_script_with_amount."""
    e = ctypes.c_int(0)
    r = lib().bitcoinconsensus_verify_script_with_amount(
        spk, len(spk) & 0xffffffff, amount, tx, len(tx) & 0xffffffff, n_in & 0xffffffff,
        flags & 0xffffffff, ctypes.byref(e))
    return r, e.value


def verify_with_flags(spent_output_script, amount, spending_transaction, input_index, flags):
    """src/lib.rs:113-139: raises ConsensusError(err) unless the spend is valid.  Lengths and the
    index are truncated to c_uint exactly as the Rust `as c_uint` casts do."""
    amount = amount - (1 << 64) if amount >= (1 << 63) else amount  # u64 -> int64 ABI slot
    ret, err = verify_script_with_amount(spent_output_script, amount, spending_transaction,
                                         input_index, flags)
    if ret != 1:
        raise ConsensusError(Error(err))


def verify(spent_output, amount, spending_transaction, input_index):
    """src/lib.rs:103-110: verify_with_flags(..., VERIFY_ALL)."""
    verify_with_flags(spent_output, amount, spending_transaction, input_index, VERIFY_ALL)


def _batch_items(items):
    """(BatchItem array, keep-alive buffers) for (spk, amount, tx, nin) tuples."""
    items = list(items)
    n = len(items)
    arr = (BatchItem * max(n, 1))()
    keep, txbufs = [], {}
    for i, (spk, amount, tx, nin) in enumerate(items):
        amount = amount - (1 << 64) if amount >= (1 << 63) else amount
        bs = ctypes.create_string_buffer(bytes(spk), max(1, len(spk)))
        tx = bytes(tx)
        bt = txbufs.get(tx)
        if bt is None:  # one buffer per distinct tx: the engine then deserializes it once
            bt = txbufs[tx] = ctypes.create_string_buffer(tx, max(1, len(tx)))
        keep.append(bs)
        arr[i] = BatchItem(ctypes.addressof(bs), len(spk), amount, ctypes.addressof(bt), len(tx),
                           nin & 0xffffffff)
    return arr, (keep, txbufs)


def verify_batch_raw(items, flags=VERIFY_ALL):
    """bitcoinconsensus_verify_batch as is: (return code, [(ret, err int)]); rc is the number of
    valid items, or -1 when the device failed (items it left unfinished carry
    ERR_DEVICE_FAILURE)."""
    arr, keep = _batch_items(items)
    n = len(keep[0])
    ret = (ctypes.c_int * max(n, 1))()
    err = (ctypes.c_int * max(n, 1))()
    rc = lib().bitcoinconsensus_verify_batch(arr, n, flags & 0xffffffff, ret, err)
    return rc, [(ret[i], err[i]) for i in range(n)]


def verify_batch(items, flags=VERIFY_ALL, device_failure="raise"):
    """items: iterable of (spent_output_script, amount, spending_transaction, input_index).
    Returns a list of (ret, Error) equal to calling the C ABI once per item; all signature work
    of the batch runs on the GPU in as few device rounds as the scripts allow.  When the device
    failed (only under DEVICE_FAILURE_ERROR) it raises RuntimeError, or with
    device_failure="mark" returns the results with DeviceFailure.ERR_DEVICE_FAILURE for the items
    left without a verdict (no verdict is ever reported for a device error)."""
    rc, res = verify_batch_raw(items, flags)
    if rc < 0 and device_failure != "mark":
        raise RuntimeError("bitcoinconsensus_verify_batch: device pipeline failed")
    return [(r, error_from_code(e)) for r, e in res]


def last_batch_stats():
    s = BatchStats()
    lib().bcc_last_batch_stats(ctypes.byref(s))
    return {k: getattr(s, k) for k, _ in BatchStats._fields_}


def debug_fail_device_rounds(rounds):
    """Fault injection (tests): the next `rounds` device rounds fail (include/bcc_amd.h)."""
    lib().bcc_debug_fail_device_rounds(rounds)


DEVICE_FAILURE_HOST, DEVICE_FAILURE_ERROR = 0, 1


def set_device_failure_policy(policy):
    """bcc_set_device_failure_policy: DEVICE_FAILURE_HOST (default) verifies a round the GPU could
    not deliver on the host CPU; DEVICE_FAILURE_ERROR reports it (-1 / abort)."""
    if lib().bcc_set_device_failure_policy(policy) != 0:
        raise ValueError(policy)


HOST_SMALL_ROUND_DEFAULT = 16  # include/bcc_amd.h BCC_HOST_SMALL_ROUND_DEFAULT


def set_host_small_round(tuples):
    """bcc_set_host_small_round: device rounds of at most `tuples` checks run on the host CPU."""
    lib().bcc_set_host_small_round(tuples)


def set_host_threads(n):
    """bcc_set_host_threads: host worker threads of a batch pass (0: the default: the affinity CPUs, or cpu_share() under a smaller cgroup quota, at most 64)."""
    L = lib()
    L.bcc_set_host_threads.argtypes = [ctypes.c_uint]
    if L.bcc_set_host_threads(n) != 0:
        raise ValueError(n)


def host_threads():
    L = lib()
    L.bcc_get_host_threads.restype = ctypes.c_uint
    return L.bcc_get_host_threads()


def cpu_share():
    """CPUs this process can keep busy: min(affinity, cgroup CPU quota) (bcc_cpu_share)."""
    L = lib()
    L.bcc_cpu_share.restype = ctypes.c_uint
    return L.bcc_cpu_share()


def set_early_q(on):
    """bcc_set_early_q: pre-extracted (key, signature) rows run their Q half on the GPU during the
    host pass of a single-chunk verify_batch call (default on)."""
    L = lib()
    L.bcc_set_early_q.argtypes = [ctypes.c_int]
    L.bcc_set_early_q(1 if on else 0)


HOST_CHAIN_BLOCKS_DEFAULT = 160  # engine.cpp g_host_chain_blocks


def set_host_chain_blocks(blocks):
    """bcc_set_host_chain_blocks: legacy checks that hash more than `blocks` blocks from their
    template midstate are hashed on the host CPU during the device round (default
    HOST_CHAIN_BLOCKS_DEFAULT; 0: every legacy chain on the GPU)."""
    L = lib()
    L.bcc_set_host_chain_blocks.argtypes = [ctypes.c_uint]
    L.bcc_set_host_chain_blocks(blocks)


def set_host_bip143_blocks(blocks):
    """bcc_set_host_bip143_blocks: BIP143 checks of a tx whose per-tx hash chains exceed `blocks`
    blocks are hashed on the host CPU (default 32; 0: every chain on the GPU)."""
    L = lib()
    L.bcc_set_host_bip143_blocks.argtypes = [ctypes.c_uint]
    L.bcc_set_host_bip143_blocks(blocks)


def set_device_key_hash(on):
    """bcc_set_device_key_hash: on an input's first run the HASH160(pubkey) == program check of a
    P2WPKH / P2PKH spend runs on the device beside the signature (default on); off: the host
    hashes every P2WPKH key before the run.  Results never depend on it."""
    L = lib()
    L.bcc_set_device_key_hash.argtypes = [ctypes.c_int]
    L.bcc_set_device_key_hash(1 if on else 0)


def set_direct_upload(on):
    """bcc_set_direct_upload: a device round's tuple rows, raw txs and sighash blobs go to HBM
    from the page-locked arrays the host pass wrote (default on); off: through one pinned image.
    Results never depend on it."""
    L = lib()
    L.bcc_set_direct_upload.argtypes = [ctypes.c_int]
    L.bcc_set_direct_upload(1 if on else 0)


def set_pipeline_chunk(items):
    """bcc_set_pipeline_chunk: verify_batch overlaps chunk k's device round with chunk k+1's host
    pass (0 disables)."""
    L = lib()
    L.bcc_set_pipeline_chunk.argtypes = [ctypes.c_size_t]
    L.bcc_set_pipeline_chunk(items)


def host_fallback_rounds():
    """Rounds verified on the host after a device failure, process-wide."""
    return lib().bcc_host_fallback_rounds()


def host_verify_tuples(pub65, msg32, r32, s32, threads=1):
    """bcc_host_verify_tuples: mi_ecdsa_verify_tuples' contract on the host CPU."""
    n = len(msg32) // 32
    out = ctypes.create_string_buffer(max(1, n))
    if lib().bcc_host_verify_tuples(pub65, msg32, r32, s32, out, n, threads) != 0:
        raise RuntimeError("bcc_host_verify_tuples failed")
    return out.raw[:n]


def set_device(device):
    lib().bcc_set_device(device)


def set_devices(devices):
    """Node sharding (include/bcc_amd.h bcc_set_devices): spread verify_batch's device rounds and
    pubkey_verify_batch(device=-1) over these GPUs ([] restores the single default device)."""
    devs = list(devices)
    arr = (ctypes.c_int * max(1, len(devs)))(*devs)
    if lib().bcc_set_devices(arr, len(devs)) != 0:
        raise ValueError(f"bad device list {devs}")


def get_devices():
    arr = (ctypes.c_int * 64)()
    n = lib().bcc_get_devices(arr, 64)
    return list(arr)[:n]


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


def _blob(parts):
    off = [0]
    for p in parts:
        off.append(off[-1] + len(p))
    return b"".join(parts), (ctypes.c_uint64 * len(off))(*off)


def pubkey_verify_batch(tuples, device=0):
    """[CPubKey(pub).Verify(hash32, der_sig) for (pub, hash32, der_sig) in tuples] as a bytes of
    0/1 (depend/bitcoin/src/pubkey.cpp:191-207): length filter + lax DER on the GPU (K_der,
    over the blobs as they are), the secp256k1 work on the GPU (include/bcc_amd.h bcc_pubkey_verify_batch).  device=-1 shards the
    tuples over the set_devices() GPUs."""
    n = len(tuples)
    if n == 0:
        return b""
    pb, po = _blob([bytes(t[0]) for t in tuples])
    sb, so = _blob([bytes(t[2]) for t in tuples])
    msg = b"".join(bytes(t[1]) for t in tuples)
    assert len(msg) == 32 * n
    out = ctypes.create_string_buffer(n)
    rc = lib().bcc_pubkey_verify_batch(pb, po, msg, sb, so, out, n, device)
    if rc != 0:
        raise RuntimeError(f"bcc_pubkey_verify_batch failed: {rc}")
    return out.raw[:n]


SIGVERSION_TAPROOT = 0
SIGVERSION_TAPSCRIPT = 1
SCRIPT_ERR_SCHNORR_SIG_SIZE = 44
SCRIPT_ERR_SCHNORR_SIG_HASHTYPE = 45
SCRIPT_ERR_SCHNORR_SIG = 46


class TaprootCheck(ctypes.Structure):
    """include/bcc_amd.h bcc_taproot_check."""
    _fields_ = [("tx", ctypes.c_char_p), ("tx_len", ctypes.c_uint),
                ("spent_outputs", ctypes.c_char_p), ("spent_outputs_len", ctypes.c_uint),
                ("n_in", ctypes.c_uint), ("sig", ctypes.c_char_p), ("sig_len", ctypes.c_uint),
                ("pubkey32", ctypes.c_char_p), ("sigversion", ctypes.c_int),
                ("annex", ctypes.c_char_p), ("annex_len", ctypes.c_uint),
                ("tapleaf_hash32", ctypes.c_char_p), ("codeseparator_pos", ctypes.c_uint32)]


def taproot_verify_batch(checks, device=0, sighashes=False, library=None):
    """GenericTransactionSignatureChecker::CheckSchnorrSignature for each check
    (depend/bitcoin/src/script/interpreter.cpp:1678-1704; include/bcc_amd.h
    bcc_taproot_verify_batch).  A check is a dict with keys tx, spent (serialized
    std::vector<CTxOut>), nin, sig, pk, sigversion and optionally annex (None: absent), tapleaf,
    codesep.  Returns [(ret, serror)] (ret -1: inputs the reference checker cannot be built for),
    plus the 32-byte sighashes when sighashes=True.  Adjacent checks of one tx should pass the
    same tx / spent bytes objects: they then share the per-tx hashes.  `library`: another build
    of the same C ABI (tests: the host code over the oracle stub)."""
    n = len(checks)
    arr = (TaprootCheck * max(n, 1))()
    keep = []
    for i, c in enumerate(checks):
        tx, spent, sig, pk = bytes(c["tx"]), bytes(c["spent"]), bytes(c["sig"]), bytes(c["pk"])
        annex = c.get("annex")
        annex = None if annex is None else bytes(annex)
        leaf = bytes(c.get("tapleaf") or bytes(32))
        if i and checks[i - 1]["tx"] is c["tx"]:
            tx = keep[-1][0]
        if i and checks[i - 1]["spent"] is c["spent"]:
            spent = keep[-1][1]
        keep.append((tx, spent, sig, pk, annex, leaf))
        assert len(pk) == 32 and len(leaf) == 32
        arr[i] = TaprootCheck(tx, len(tx), spent, len(spent), c["nin"], sig, len(sig), pk,
                              c.get("sigversion", SIGVERSION_TAPROOT),
                              annex, 0 if annex is None else len(annex), leaf,
                              c.get("codesep", 0xFFFFFFFF))
    ret = (ctypes.c_int * max(n, 1))()
    err = (ctypes.c_int * max(n, 1))()
    hs = ctypes.create_string_buffer(32 * max(n, 1)) if sighashes else None
    L = library if library is not None else lib()
    rc = L.bcc_taproot_verify_batch(arr, n, ret, err, hs, device)
    if rc != 0:
        raise RuntimeError(f"bcc_taproot_verify_batch failed: {rc}")
    out = [(ret[i], err[i]) for i in range(n)]
    if sighashes:
        return out, [hs.raw[32 * i: 32 * i + 32] for i in range(n)]
    return out


class TupleSet:
    """Synthetic signature tuples staged in HBM (include/bcc_amd.h, bcc_tupleset_*).

    kind "c4": n ECDSA (pub, msg32, DER sig) tuples, 90 % valid + 18 adversarial classes.
    kind "c5": n BIP340 rows; `vectors` = [(sig64, msg32, xonly32, expected)] tiled in."""

    C4_CLASSES = ("valid", "flip_r", "flip_s", "flip_msg", "high_s", "r_ge_n", "s_ge_n", "r_zero",
                  "s_zero", "r_overlong", "r_zeropad", "pub_no_sqrt", "pub_x_ge_p",
                  "pub_04_bad_y", "pub_04", "pub_hybrid_ok", "pub_hybrid_bad", "pub_bad_header",
                  "wrong_key")

    def __init__(self, n, kind="c4", seed=None, device=0, vectors=(), first=0, total=None):
        """Rows [first, first + n) of the global set of `total` rows (default: n) from `seed`."""
        L = blib()
        total = first + n if total is None else total
        if kind == "c4":
            self.h = L.bcc_tupleset_c4_range(n, 0x5EED0004 if seed is None else seed, first,
                                             total, device)
        elif kind == "c5":
            v = list(vectors)
            self.h = L.bcc_tupleset_c5_range(n, 0x5EED0005 if seed is None else seed, first,
                                             b"".join(x[0] for x in v), b"".join(x[1] for x in v),
                                             b"".join(x[2] for x in v), bytes(int(x[3]) for x in v),
                                             len(v), device)
        else:
            raise ValueError(kind)
        if not self.h:
            raise RuntimeError(f"bcc_tupleset_{kind} failed")
        self.kind, self.n = kind, n

    def run(self, stream=None):
        rc = blib().bcc_tupleset_run(self.h, stream)
        if rc != 0:
            raise RuntimeError(f"bcc_tupleset_run failed: {rc}")

    def verdicts(self):
        out = ctypes.create_string_buffer(max(self.n, 1))
        if blib().bcc_tupleset_verdicts(self.h, out) != 0:
            raise RuntimeError("bcc_tupleset_verdicts failed")
        return out.raw[: self.n]

    def host(self):
        """numpy views of the host inputs: dict with msg32, cls, expect and pub/sig blobs +
        offsets (c4) or sig64/xonly32 (c5).  Valid while the set lives."""
        import numpy as np
        v = TuplesetHost()
        blib().bcc_tupleset_view(self.h, ctypes.byref(v))
        n = v.n

        def arr(ptr, count, dt=np.uint8):
            if not ptr:
                return None
            c = ctypes.c_uint64 if dt == np.uint64 else ctypes.c_uint8
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(c)), shape=(count,))

        d = dict(msg32=arr(v.msg32, 32 * n), cls=arr(v.cls, n), expect=arr(v.expect, n))
        if self.kind == "c4":
            d["pub_off"] = arr(v.pub_off, n + 1, np.uint64)
            d["sig_off"] = arr(v.sig_off, n + 1, np.uint64)
            d["pub_blob"] = arr(v.pub_blob, int(d["pub_off"][-1]))
            d["sig_blob"] = arr(v.sig_blob, int(d["sig_off"][-1]))
        else:
            d["sig64"] = arr(v.sig64, 64 * n)
            d["xonly32"] = arr(v.xonly32, 32 * n)
        return d

    def tuple(self, i):
        d = self.host()
        if self.kind == "c4":
            po, so = d["pub_off"], d["sig_off"]
            return (d["pub_blob"][po[i]:po[i + 1]].tobytes(), d["msg32"][32 * i:32 * i + 32].tobytes(),
                    d["sig_blob"][so[i]:so[i + 1]].tobytes())
        return (d["sig64"][64 * i:64 * i + 64].tobytes(), d["msg32"][32 * i:32 * i + 32].tobytes(),
                d["xonly32"][32 * i:32 * i + 32].tobytes())

    def free(self):
        if self.h:
            blib().bcc_tupleset_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def ecdsa_verify_tuples(pub65, msg32, r32, s32, device=0):
    """Inner tuple ABI: n tuples as concatenated byte strings -> bytes of verdicts (0/1)."""
    n = len(msg32) // 32
    assert len(pub65) == 65 * n and len(r32) == 32 * n and len(s32) == 32 * n
    out = ctypes.create_string_buffer(max(n, 1))
    rc = lib().mi_ecdsa_verify_tuples(pub65, msg32, r32, s32, out, n, device)
    if rc != 0:
        raise RuntimeError(f"mi_ecdsa_verify_tuples failed: hip error {rc}")
    return out.raw[:n]


def schnorr_verify_tuples(sig64, msg32, xonly32, device=0):
    """BIP340 tuple ABI (config C5): n rows as concatenated byte strings -> bytes of verdicts.
    Row semantics of secp256k1_xonly_pubkey_parse + secp256k1_schnorrsig_verify."""
    n = len(msg32) // 32
    assert len(sig64) == 64 * n and len(xonly32) == 32 * n
    out = ctypes.create_string_buffer(max(n, 1))
    rc = lib().mi_schnorr_verify_tuples(sig64, msg32, xonly32, out, n, device)
    if rc != 0:
        raise RuntimeError(f"mi_schnorr_verify_tuples failed: hip error {rc}")
    return out.raw[:n]


def schnorr_verify_device(d_sig64, d_msg32, d_xonly32, d_verdict, n, stream=None):
    """Device-pointer BIP340 entry (pointers as ints, e.g. torch tensor data_ptr())."""
    rc = lib().mi_schnorr_verify_device(d_sig64, d_msg32, d_xonly32, d_verdict, n, stream)
    if rc != 0:
        raise RuntimeError(f"mi_schnorr_verify_device failed: hip error {rc}")


def gen_schnorr_sign(d32, m32, k32, device=0):
    """Synthetic-input generator: BIP340 (sig64, xonly32, ok) for n (d, m, nonce) rows."""
    n = len(d32) // 32
    sig = ctypes.create_string_buffer(64 * max(n, 1))
    xo = ctypes.create_string_buffer(32 * max(n, 1))
    ok = ctypes.create_string_buffer(max(n, 1))
    rc = blib().mi_gen_schnorr_sign(d32, m32, k32, n, sig, xo, ok, device)
    if rc != 0:
        raise RuntimeError(f"mi_gen_schnorr_sign failed: hip error {rc}")
    return sig.raw[: 64 * n], xo.raw[: 32 * n], ok.raw[:n]


def release_thread_state():
    """Frees the calling thread's cached host / device state (bcc_release_thread_state)."""
    lib().bcc_release_thread_state()


def debug_scratch_cap_lanes(lanes):
    """Test hook: signature-kernel scratch requests above `lanes` lanes fail as out of memory
    (0: no cap); the library then halves its chunk until it fits (bcc_amd.h)."""
    lib().bcc_debug_scratch_cap_lanes(lanes)


def set_chunk_lanes(lanes):
    """Lanes per signature-kernel launch (0 restores the default); results never depend on it."""
    lib().bcc_set_chunk_lanes(ctypes.c_size_t(lanes))


def microbench_sustained(op, waves_per_simd=8, target_ms=20.0, warm_s=1.0, reps=5):
    """Sustained issue rate of microbenchmark `op` (lane-instructions/s), the in-kernel clock it
    ran at (GHz) and the launch time (ms): mi_microbench_sustained."""
    r, c, m = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_double(0)
    rc = blib().mi_microbench_sustained(op, waves_per_simd, target_ms, warm_s, reps,
                                        ctypes.byref(r), ctypes.byref(c), ctypes.byref(m))
    if rc != 0:
        raise RuntimeError(f"mi_microbench_sustained failed: {rc}")
    return r.value, c.value, m.value


def primbench(prim, iters=4096, warm=3):
    """(cycles per primitive per wave at 4 waves/SIMD, launch ms): mi_primbench."""
    c, m = ctypes.c_double(0), ctypes.c_double(0)
    rc = blib().mi_primbench(prim, iters, warm, ctypes.byref(c), ctypes.byref(m))
    if rc != 0:
        raise RuntimeError(f"mi_primbench failed: {rc}")
    return c.value, m.value


def microbench(op, iters=4096):
    r = ctypes.c_double(0)
    rc = blib().mi_microbench(op, iters, ctypes.byref(r))
    if rc != 0:
        raise RuntimeError(f"mi_microbench failed: {rc}")
    return r.value
