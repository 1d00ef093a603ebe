import ctypes, os, random
HERE = os.path.dirname(os.path.abspath(__file__))
L = ctypes.CDLL(os.path.join(HERE, "fe_ilp.so"))
nb = 2048
lanes = nb * 256
rng = random.Random(5)
buf = b"".join(rng.randbytes(32) for _ in range(4 * lanes))
outs = {}
for m in (0, 1, 2, 3):
    out = ctypes.create_string_buffer(len(buf))
    r = ctypes.c_double()
    rc = L.fe_ilp(m, 1000, buf, out, nb, ctypes.byref(r))
    outs[m] = out.raw
    print(f"mode {m}: rc {rc} {r.value / 1e9:.1f} G modmul/s", flush=True)
print("dual == single (2 chains):", outs[0] == outs[1], " (4 chains):", outs[2] == outs[3])
