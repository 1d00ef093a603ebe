"""CPU: the C-ABI library loads (no GPU needed) and exports every function include/*.h declares;
the Python mirror exposes the Rust crate's API surface (src/lib.rs)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "rust-bitcoinconsensus_amd", "librbc_amd.so")
BENCH_LIB = os.path.join(ROOT, "rust-bitcoinconsensus_amd", "librbc_bench.so")


def declared_functions(headers=("bitcoinconsensus.h", "bcc_amd.h")):
    names = set()
    for h in headers:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", src):
            names.add(m.group(1))
    return names - {"sizeof"}


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(LIB), "-j8"])
    return ctypes.CDLL(LIB)


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert {"bitcoinconsensus_verify_script", "bitcoinconsensus_verify_script_with_amount",
            "bitcoinconsensus_version", "bitcoinconsensus_verify_batch",
            "mi_ecdsa_verify_tuples"} <= names
    missing = [n for n in sorted(names) if not hasattr(lib, n)]
    assert not missing, missing


def test_bench_library_exports_its_header():
    """librbc_bench.so (synthetic workloads / generators / microbenchmark, include/bcc_bench.h)
    exports everything its header declares; the product library exports none of it."""
    if not os.path.exists(BENCH_LIB):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(LIB), "-j8"])
    b = ctypes.CDLL(BENCH_LIB)
    p = ctypes.CDLL(LIB)
    names = declared_functions(("bcc_bench.h",))
    assert {"bcc_workload_p2wpkh", "bcc_workload_from_items", "bcc_tupleset_c4",
            "mi_microbench"} <= names
    assert not [n for n in sorted(names) if not hasattr(b, n)]
    assert not [n for n in sorted(names) if hasattr(p, n)]


def test_source_hash_matches_tree(lib):
    """Provenance: the library embeds the hash of the sources it was built from."""
    import sys
    sys.path.insert(0, os.path.dirname(LIB))
    from source_hash import source_hash
    lib.bcc_source_hash.restype = ctypes.c_char_p
    assert lib.bcc_source_hash().decode() == source_hash()


def test_version_and_flag_check_need_no_gpu(lib):
    assert lib.bitcoinconsensus_version() == 1
    e = ctypes.c_int(-1)
    # invalid flags are rejected before any device work (bitcoinconsensus.cpp:83-85)
    assert lib.bitcoinconsensus_verify_script_with_amount(b"", 0, ctypes.c_int64(0), b"", 0, 0,
                                                          0xE16, ctypes.byref(e)) == 0
    assert e.value == 5
    assert lib.bitcoinconsensus_verify_script(b"", 0, b"", 0, 0, 0x800, ctypes.byref(e)) == 0
    assert e.value == 4  # ERR_AMOUNT_REQUIRED


def test_python_mirror_api_surface():
    import bitcoinconsensus_amd as B
    assert B.VERIFY_ALL == 0xE15
    assert [e.value for e in B.Error] == [0, 1, 2, 3, 4, 5]
    assert B.height_to_flags(0) == 0
    assert B.height_to_flags(173805) == B.VERIFY_P2SH
    assert B.height_to_flags(481824) == B.VERIFY_ALL
    for name in ("verify", "verify_with_flags", "verify_batch", "version", "height_to_flags"):
        assert callable(getattr(B, name))


def test_python_structs_match_c_layout(tmp_path):
    """The ctypes mirrors of the ABI's structs have the C sizes (a short mirror would let the
    library write past the Python buffer)."""
    import bitcoinconsensus_amd as B
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "bcc_bench.h"\n'
                   'int main(void) { printf("%zu %zu %zu %zu %zu\\n",'
                   ' sizeof(bcc_batch_stats), sizeof(bcc_batch_item), sizeof(bcc_tupleset_host),'
                   ' sizeof(bcc_taproot_check), offsetof(bcc_taproot_check, codeseparator_pos));'
                   ' return 0; }\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    assert got == [ctypes.sizeof(B.BatchStats), ctypes.sizeof(B.BatchItem),
                   ctypes.sizeof(B.TuplesetHost), ctypes.sizeof(B.TaprootCheck),
                   B.TaprootCheck.codeseparator_pos.offset]


def test_device_failure_code_through_verify_batch_raw():
    """BCC_DEVICE_FAILURE_ERROR through the product library's verify_batch (no GPU needed: every
    device round is made to fail): rc == -1, items that needed a signature verdict carry err 6
    (BCC_ERR_DEVICE_FAILURE), and the Python mapping turns 6 into DeviceFailure, never into the
    crate's Error (lib.rs:172-185 has discriminants 0-5 only; INTEGRATION.md binds err_out as
    c_int for that reason)."""
    import sys
    code = f"""
import sys
sys.path[:0] = [{os.path.dirname(LIB)!r}, {os.path.join(ROOT, 'tests')!r}]
import bitcoinconsensus_amd as B
from fixtures import load_json
vs = [v for v in load_json("crate_vectors.json") if v["flags"] == 0xE15]
items = [(bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"]) for v in vs]
B.set_device_failure_policy(B.DEVICE_FAILURE_ERROR)
B.set_host_small_round(0)
B.debug_fail_device_rounds(1 << 20)
rc, res = B.verify_batch_raw(items)
assert rc == -1, rc
for v, (r, e) in zip(vs, res):
    assert r == 0
    assert e == 6 if v["ret"] == 1 else e in (6, v["err"]), (v["name"], e)
marked = B.verify_batch(items, device_failure="mark")
assert [int(e) for _, e in marked] == [e for _, e in res]
assert all(isinstance(e, B.DeviceFailure) for (_, e), (_, c) in zip(marked, res) if c == 6)
try:
    B.verify_batch(items)
    raise SystemExit("no RuntimeError")
except RuntimeError:
    pass
for c in range(6):
    assert B.error_from_code(c) is B.Error(c)
try:
    B.error_from_code(7)
    raise SystemExit("no ValueError")
except ValueError:
    pass
print("ok")
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, (p.returncode, p.stdout, p.stderr[-2000:])


def test_workload_accessors_pass_row_capacity(monkeypatch):
    """Host logic of the bench library's row accessors (no GPU: the library is a stub object):
    Workload.verdicts / msgs / tuple_items size their buffers by staged tuple ROWS (a block
    workload's multisig inputs have several) and pass that capacity to the C entry points, which
    refuse a short buffer (include/bcc_bench.h BCC_BENCH_ERR_CAPACITY) instead of writing past it;
    a refusal surfaces as RuntimeError."""
    import ctypes
    import sys
    sys.path.insert(0, os.path.dirname(LIB))
    import bitcoinconsensus_amd as B
    rows, seen = 7, {}

    class Stub:
        def _check(self, name, need, out, cap):
            seen[name] = (cap, ctypes.sizeof(out))
            assert cap <= ctypes.sizeof(out)
            return -2 if cap < need else 0

        def bcc_workload_verdicts(self, h, out, cap):
            return self._check("verdicts", rows, out, cap)

        def bcc_workload_msgs(self, h, out, cap):
            return self._check("msgs", 32 * rows, out, cap)

        def bcc_workload_tuple_items(self, h, out, cap):
            seen["tuple_items"] = (cap, len(out))
            return -2 if cap < rows else 0

    w = B.Workload.__new__(B.Workload)
    w.h = None
    monkeypatch.setattr(B, "blib", lambda: Stub())
    monkeypatch.setattr(B.Workload, "shape", lambda self: {"tuples": rows})
    monkeypatch.setattr(B.Workload, "__del__", lambda self: None, raising=False)
    assert len(w.verdicts()) == rows and seen["verdicts"] == (rows, rows)
    assert len(w.msgs()) == 32 * rows and seen["msgs"] == (32 * rows, 32 * rows)
    assert len(w.tuple_items()) == rows and seen["tuple_items"] == (rows, rows)
    monkeypatch.setattr(B.Workload, "shape", lambda self: {"tuples": rows - 1})
    for f in (w.verdicts, w.msgs, w.tuple_items):
        with pytest.raises(RuntimeError):
            f()


def test_host_rounds_without_gpu_through_the_page_locked_pool():
    """The product library's verify_batch with every round on the host lane code, on a machine
    without a GPU: the interpreter's rows and blobs come from the page-locked pool
    (pipeline.h pinned_alloc), which falls back to ordinary memory when the runtime cannot pin;
    results equal the crate vectors' before and after bcc_release_thread_state hands the pool's
    blocks back (pinned_trim) and across repeated calls that reuse them."""
    import sys
    code = f"""
import sys
sys.path[:0] = [{os.path.dirname(LIB)!r}, {os.path.join(ROOT, 'tests')!r}]
import bitcoinconsensus_amd as B
from fixtures import load_json
vs = [v for v in load_json("crate_vectors.json")] * 300
items = [(bytes.fromhex(v["spk"]), v["amount"], bytes.fromhex(v["tx"]), v["nin"]) for v in vs]
B.set_host_small_round(1 << 30)
for rep in range(3):
    for flags in sorted(set(v["flags"] for v in vs)):
        idx = [i for i, v in enumerate(vs) if v["flags"] == flags]
        got = B.verify_batch([items[i] for i in idx], flags)
        for i, (r, e) in zip(idx, got):
            assert r == vs[i]["ret"], (vs[i]["name"], r)
            assert r == 1 or int(e) == vs[i]["err"], (vs[i]["name"], int(e))
    if rep == 1:
        B.release_thread_state()
print("ok")
"""
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, (p.returncode, p.stdout, p.stderr[-2000:])
