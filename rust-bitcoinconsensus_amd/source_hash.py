"""Hash of the sources librbc_amd.so / librbc_bench.so are built from (provenance check).

The Makefile embeds it into both libraries (bcc_source_hash()); __graft_entry__.smoke() and
bench.py recompute it from the tree and refuse a library built from other sources.
    python source_hash.py        prints the hash
"""
import hashlib
import os

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
EXTS = (".h", ".hip", ".cpp")


def source_files():
    out = []
    for base in (os.path.join(PKG, "csrc"), os.path.join(ROOT, "include")):
        for d, _, fs in os.walk(base):
            out += [os.path.join(d, f) for f in fs if f.endswith(EXTS)]
    out.append(os.path.join(PKG, "Makefile"))
    return sorted(out, key=lambda p: os.path.relpath(p, ROOT).replace(os.sep, "/"))


def source_hash():
    h = hashlib.sha256()
    for p in source_files():
        rel = os.path.relpath(p, ROOT).replace(os.sep, "/")
        h.update(rel.encode() + b"\0" + hashlib.sha256(open(p, "rb").read()).hexdigest().encode()
                 + b"\n")
    return h.hexdigest()


if __name__ == "__main__":
    print(source_hash())
