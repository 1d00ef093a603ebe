"""Runs tools/fe9/ubench2.hip on the GPU: issue rates (T lane-instr/s) and dependent latencies."""
import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "fe9", "_build", "ubench2.so"))
T = ["mad same-sgpr", "mad distinct-sgpr", "addc_e64 distinct", "add_co_e64 distinct", "and",
     "mov", "sub_u32", "lshlrev_b32", "add3", "lshl_add_u32", "bfe", "lshrrev_b64",
     "mad+addc distinct"]
LT = ["mad dep", "add_u32 dep", "lshrrev_b64 dep", "mad->shr64 dep (pair)", "add_co->addc dep (pair)", "and dep",
      "add_u32 indep (lone wave)", "mad indep (lone wave)"]
for op, name in enumerate(T):
    r = ctypes.c_double()
    L.ub_throughput(op, 2048, ctypes.byref(r))
    print(f"thr {name:24s} {r.value / 1e12:6.2f} T/s", flush=True)
for op, name in enumerate(LT):
    r = ctypes.c_double()
    L.ub_latency(op, 4096, ctypes.byref(r))
    print(f"lat {name:24s} {r.value:6.2f} ticks/instr", flush=True)
