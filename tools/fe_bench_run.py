"""Dev tool: run tools/_build/fe_bench.so variants on the GPU; cross-check asm vs portable."""
import ctypes, os, random, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "fe_bench.so"))
nb = 1024
lanes = nb * 256
rng = random.Random(3)
buf = b"".join(rng.randbytes(32) for _ in range(2 * lanes))
res = {}
for sq in (0, 1):
    outs = []
    for v in (0, 1, 2, 3):
        out = ctypes.create_string_buffer(len(buf))
        r = ctypes.c_double()
        L.fe_bench(v, sq, 2000, buf, out, nb, ctypes.byref(r))
        outs.append(out.raw)
        print(f"{'sqr' if sq else 'mul'} variant {v}: {r.value/1e9:.1f} G lane-ops/s", flush=True)
    print("  asm == portable:", outs[0] == outs[1], " col == portable:", outs[0] == outs[2], " r29 == portable:", outs[0] == outs[3])
