"""Instruction-class histogram of one kernel in a gfx950 assembly listing, per basic block.

    python3 tools/isa/isa_blocks.py ev.s twist_ladder_kernelILb0 [--blocks]

Classes: mad64 (v_mad_u64_u32), addc (v_addc_co_u32 / v_add_co_u32 / v_sub*_co*), add (v_add_u32,
v_add3_u32, v_sub_u32, ...), cndmask, mov (v_mov*), logic (and/or/xor/not/bfi/alignbit/lshl*),
mul32 (v_mul_lo/hi), other VALU, VMEM (global_/buffer_/flat_), LDS (ds_), SMEM (s_load*), SALU,
branch, wait (s_waitcnt), nop.  Loops are reported from backward branches.  The rare asm fold tails (skipped by a wave-uniform
s_cbranch_scc0 .LdoneN unless a lane needs them) are left out unless --all-static."""
import re
import sys
from collections import Counter, OrderedDict


def klass(op):
    if op.startswith("v_mad_u64_u32") or op.startswith("v_mad_i64_i32"):
        return "mad64"
    if re.match(r"v_(add|sub|subrev)c?_co_u32", op) or op.startswith("v_addc") or op.startswith("v_subb"):
        return "addc"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith("v_mov") or op.startswith("v_readfirstlane") or op.startswith("v_writelane") \
            or op.startswith("v_readlane"):
        return "mov"
    if re.match(r"v_(add|sub|subrev|add3|lshl_add|add_lshl|min|max)_u32|v_(add|sub)_u16|v_lshl_add_u64", op):
        return "add"
    if re.match(r"v_(and|or|xor|not|bfi|bfe|alignbit|alignbyte|lshl|lshr|ashr|perm|and_or|or3|xad|lshlrev|lshrrev|ashrrev)", op):
        return "logic"
    if re.match(r"v_mul_(lo|hi)_u32|v_mul_u32_u24|v_mad_u32_u24", op):
        return "mul32"
    if re.match(r"v_cmp", op):
        return "cmp"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


EXACT_STATIC = "--all-static" in sys.argv


def parse(path, name):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", l))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = dict(c=Counter(), succ=[], n=0)
    order = [cur]
    skip_to = None  # inside an asm fold tail behind a wave-uniform branch (rarely executed)
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        if skip_to:
            if l.strip().startswith(skip_to + ":"):
                skip_to = None
            continue
        m = re.search(r"s_cbranch_scc0\s+(\.Ldone\d+)", l)
        if m and not EXACT_STATIC:
            skip_to = m.group(1)
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            prev = cur
            cur = m.group(1)
            blocks[cur] = dict(c=Counter(), succ=[], n=0)
            order.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        k = klass(op)
        blocks[cur]["c"][k] += 1
        blocks[cur]["n"] += 1
        if k == "branch":
            t = re.search(r"(\.LBB\d+_\d+)", s)
            if t:
                blocks[cur]["succ"].append(t.group(1))
        blocks[cur].setdefault("ops", Counter())[op] += 1
    return blocks, order


def main():
    path, name = sys.argv[1], sys.argv[2]
    blocks, order = parse(path, name)
    pos = {b: i for i, b in enumerate(order)}
    tot = Counter()
    for b in order:
        tot += blocks[b]["c"]
    print(f"{name}: {len(order)} blocks, {sum(tot.values())} instructions")
    print("  total:", dict(tot.most_common()))
    loops = []
    for b in order:
        for s in blocks[b]["succ"]:
            if s in pos and pos[s] <= pos[b]:
                loops.append((s, b))
    for head, tail in loops:
        c = Counter()
        for b in order[pos[head]:pos[tail] + 1]:
            c += blocks[b]["c"]
        print(f"  loop {head}..{tail} ({pos[tail] - pos[head] + 1} blocks, {sum(c.values())} instr):",
              dict(c.most_common()))
    if "--blocks" in sys.argv:
        for b in order:
            if blocks[b]["n"] >= 50:
                print(f"  {b}: {blocks[b]['n']}", dict(blocks[b]["c"].most_common(8)), "->",
                      blocks[b]["succ"])


if __name__ == "__main__":
    main()
