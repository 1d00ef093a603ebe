"""Runs tools/fe9/fe9_bench.hip builds (one per BCC_FE9_CHAIN variant) on the GPU: group-law
throughput radix 2^29 vs 2^32 and a cross-check of the resulting points (same formulas -> same
Jacobian coordinates mod p).  Usage: python tools/fe9/run.py [variants...]"""
import ctypes
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
P = 2**256 - 2**32 - 977
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8


def limbs(x):
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def main():
    variants = sys.argv[1:] or ["0", "1", "2"]
    nblocks, lanes = 4096, 4096 * 256
    rng = random.Random(5)
    # points: a = (k G) in Jacobian with random Z, b = affine-ish (x, y, zinv) random field values
    # (throughput only; the cross-check compares radix 2^29 with radix 2^32 on the same inputs)
    base = []
    for i in range(lanes):
        z = rng.randrange(1, P)
        base += [GX * z * z % P, GY * z * z * z % P, z, rng.randrange(P), rng.randrange(P),
                 rng.randrange(1, P)]
    raw = b"".join(b"".join(v.to_bytes(4, "little") for v in limbs(x)) for x in base)
    for v in variants:
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "fe9", "_build", f"fe9_bench_{v}.so"))
        L.fe9_bench.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_double)]
        res = {}
        outs = {}
        for op, name, it in ((0, "dbl29", 64), (1, "dbl32", 64), (2, "add29", 32), (3, "add32", 32)):
            buf = ctypes.create_string_buffer(raw, len(raw))
            r = ctypes.c_double()
            assert L.fe9_bench(op, it, buf, nblocks, ctypes.byref(r)) == 0  # warm + check run
            outs[name] = buf.raw
            buf2 = ctypes.create_string_buffer(raw, len(raw))
            assert L.fe9_bench(op, it * 4, buf2, nblocks, ctypes.byref(r)) == 0
            res[name] = r.value / 1e6
        def canon(b):
            xs = [int.from_bytes(b[32 * i:32 * i + 32], "little") % P for i in range(len(b) // 32)]
            return [x for j, x in enumerate(xs) if j % 6 < 3]
        same_d = canon(outs["dbl29"]) == canon(outs["dbl32"])
        same_a = canon(outs["add29"]) == canon(outs["add32"])
        print(f"chain {v}: " + "  ".join(f"{k} {x:8.1f} M/s" for k, x in res.items()) +
              f"  | dbl 29/32 {res['dbl29'] / res['dbl32']:.3f}  add 29/32 {res['add29'] / res['add32']:.3f}"
              f"  | identical results: dbl {same_d} add {same_a}", flush=True)


if __name__ == "__main__":
    main()
