"""Quick on-box probe: integer-ALU microbenchmarks + ECDSA kernel throughput (dev tool)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-bitcoinconsensus_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa
import torch  # noqa
import bitcoinconsensus_amd as B  # noqa
from fixtures import ecdsa_tuples, pub_to_tuple  # noqa
from oracle_ctypes import Oracle  # noqa

out = {}
names = ["mad_u64_u32", "mul_lo_u32", "mul_hi_u32", "add_co_u32", "addc_co_u32", "mad_u32_u24",
         "lshl_add_u64", "fma_f64", "add_u32"]
if "--ubench" in sys.argv:
    for op, nm in enumerate(names):
        r = B.microbench(op, 4096)
        out[nm] = r / 1e12
        print(f"{nm:14s} {r/1e12:8.2f} T lane-ops/s", flush=True)

O = Oracle()
ts = [t for t in ecdsa_tuples() if t["verdict"] == 1]
n = int(os.environ.get("PROBE_N", "262144"))
tag = np.zeros(n, np.uint8)
arr = {k: np.zeros((n, 32), np.uint8) for k in "xyrsm"}
base = []
for t in ts:
    tg, x, y = pub_to_tuple(t["pub"])
    ok, r, s = O.der_parse_lax(t["sig"])
    base.append((tg, x, y, r, s, t["hash"]))
for i in range(n):
    tg, x, y, r, s, m = base[i % len(base)]
    tag[i] = tg
    for k, v in zip("xyrsm", (x, y, r, s, m)):
        arr[k][i] = np.frombuffer(v, np.uint8)
dev = torch.device("cuda:0")
d = {k: torch.from_numpy(v).to(dev) for k, v in arr.items()}
dtag = torch.from_numpy(tag).to(dev)
dv = torch.zeros(n, dtype=torch.uint8, device=dev)
stream = torch.cuda.current_stream().cuda_stream
L = B.lib()


def run():
    rc = L.mi_ecdsa_verify_device(dtag.data_ptr(), d["x"].data_ptr(), d["y"].data_ptr(),
                                  d["r"].data_ptr(), d["s"].data_ptr(), d["m"].data_ptr(),
                                  dv.data_ptr(), n, stream)
    assert rc == 0, rc


run()
torch.cuda.synchronize()
valid = int(dv.sum().item())
print("valid", valid, "of", n, flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(3):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 3
print(f"ecdsa kernel: {ms:.2f} ms for {n} -> {n/ms/1e3:.3f} M verifies/s", flush=True)
out["verify_per_s"] = n / ms * 1e3
out["valid"] = valid
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "probe.json"), "w"), indent=1)
