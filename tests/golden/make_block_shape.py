"""Shape of the reference's benchmark block (config C3's histogram), run in the build container.

    python3 tests/golden/make_block_shape.py

Reads depend/bitcoin/src/bench/data/block413567.raw (the block the reference's own
bench/checkblock.cpp deserializes) and records, per non-coinbase transaction, its input and output
counts and the script type of each output.  Only these counts travel (block413567_shape.json):
the C3 workload generator re-creates transactions of exactly this shape with synthetic keys,
because the block's prevouts (and so its spent scripts and amounts) are not in the block.
"""
import json
import os

SRC = "/root/reference/depend/bitcoin/src/bench/data/block413567.raw"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "block413567_shape.json")


def main():
    b = open(SRC, "rb").read()
    pos = 80

    def cs():
        nonlocal pos
        v = b[pos]
        pos += 1
        if v < 0xFD:
            return v
        k = {0xFD: 2, 0xFE: 4, 0xFF: 8}[v]
        v = int.from_bytes(b[pos:pos + k], "little")
        pos += k
        return v

    ntx = cs()
    txs, scriptsig_lens, out_types = [], [], {}
    for t in range(ntx):
        pos += 4
        seg = b[pos] == 0 and b[pos + 1] == 1
        if seg:
            pos += 2
        nin = cs()
        for _ in range(nin):
            pos += 36
            n = cs()
            if t:
                scriptsig_lens.append(n)
            pos += n + 4
        nout = cs()
        for _ in range(nout):
            pos += 8
            n = cs()
            spk = b[pos:pos + n]
            kind = ("p2pkh" if n == 25 and spk[0] == 0x76 else "p2sh" if n == 23 and spk[0] == 0xA9
                    else "other")
            out_types[kind] = out_types.get(kind, 0) + 1
            pos += n
        if seg:
            for _ in range(nin):
                for _ in range(cs()):
                    pos += cs()
        pos += 4
        if t:
            txs.append([nin, nout])
    assert pos == len(b), (pos, len(b))
    scriptsig_lens.sort()
    json.dump(dict(source="block413567.raw (reference bench/data)", transactions=ntx,
                   non_coinbase=len(txs), inputs=sum(t[0] for t in txs),
                   max_inputs=max(t[0] for t in txs),
                   median_scriptsig=scriptsig_lens[len(scriptsig_lens) // 2],
                   output_types=out_types, txs=txs), open(OUT, "w"))
    print(f"{ntx} txs, {sum(t[0] for t in txs)} inputs, max {max(t[0] for t in txs)} -> {OUT}")


if __name__ == "__main__":
    main()
