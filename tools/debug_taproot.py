"""Debug: Taproot golden cases on the GPU, every sighash mismatch with its neighbours and the same
case run alone / in a small window.   python tools/debug_taproot.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rust-bitcoinconsensus_amd"), os.path.join(ROOT, "tests")]
import bitcoinconsensus_amd as B  # noqa: E402
from fixtures import taproot_checks  # noqa: E402

cases = taproot_checks()
out, hs = B.taproot_verify_batch(cases, sighashes=True)
bad = []
for i, ((ret, serr), h, c) in enumerate(zip(out, hs, cases)):
    want = c["sighash"] if c["sighash"] is not None else bytes(32)
    if ret != -1 and h != want:
        bad.append(i)
print("mismatching sighashes:", len(bad), bad[:30])
where = {h: i for i, h in enumerate(hs)}
exp_where = {c["sighash"]: i for i, c in enumerate(cases) if c["sighash"]}
for i in bad[:6]:
    c = cases[i]
    print(i, c["cls"], "ret", out[i], "got", hs[i].hex()[:16], "want", (c["sighash"] or b"").hex()[:16],
          "got==want of case", exp_where.get(hs[i]), "pk", c["pk"].hex()[:8])
    o1, h1 = B.taproot_verify_batch([c], sighashes=True)
    print("   alone:", o1, h1[0].hex()[:16], "ok" if h1[0] == c["sighash"] else "BAD")
    lo = max(0, i - 3)
    o2, h2 = B.taproot_verify_batch(cases[lo:i + 3], sighashes=True)
    print("   window:", ["ok" if h2[k] == (cases[lo + k]["sighash"] or bytes(32)) or o2[k][0] == -1 else "BAD"
                         for k in range(len(h2))])
    c2 = dict(c)
    c2["pk"] = cases[[k for k, x in enumerate(cases) if x["cls"] == "valid"][0]]["pk"]
    o3, h3 = B.taproot_verify_batch([c2], sighashes=True)
    print("   with a valid key:", o3, "ok" if h3[0] == c["sighash"] else "BAD")
