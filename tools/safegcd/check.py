"""Checks tools/safegcd/proto.cpp against pow(a, -1, m) for secp256k1's p and n: random and edge
operands; prints the batch-count distribution (30 divsteps per batch)."""
import collections
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
P = 2**256 - 2**32 - 977
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141


def main():
    exe = os.path.join(HERE, "proto")
    subprocess.check_call(["g++", "-O2", "-o", exe, os.path.join(HERE, "proto.cpp")])
    rng = random.Random(1)
    cases = []
    for m in (P, N):
        cases += [(m, a) for a in (1, 2, 3, m - 1, m - 2, (m + 1) // 2, 2**255 % m, 2**200)]
        cases += [(m, rng.randrange(1, m)) for _ in range(20000)]
    inp = "".join(f"{m:064x} {a:064x}\n" for m, a in cases)
    out = subprocess.run([exe], input=inp, capture_output=True, text=True, check=True).stdout.split("\n")
    bad, hist = 0, collections.Counter()
    for (m, a), line in zip(cases, out):
        r, b = line.split()
        hist[int(b)] += 1
        if int(r, 16) != pow(a, -1, m):
            bad += 1
    print("mismatches", bad, "of", len(cases), "batches", sorted(hist.items()))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
