"""Static per-basic-block instruction mix of one kernel in a hipcc -S listing.

usage: python tools/isa_blocks.py file.s KERNEL_SUBSTRING [--min N]

Prints, for every basic block of the kernel with at least N instructions, its label, the
instruction count by class (v_mad_u64_u32 / other VALU / LDS / global / SALU+branch) and whether
it ends in a backward branch (a loop latch).  Used to count the non-multiply instructions of the
NTT butterflies."""
import re
import sys


def classify(op):
    if op.startswith("v_mad_u64_u32"):
        return "mad64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_waitcnt", "s_barrier", "s_nop")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 20
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*%s\S*:" % re.escape(name), l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    blocks, cur, order = {}, "entry", ["entry"]
    blocks[cur] = []
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        blocks[cur].append(t.split()[0] if " " in t else t)
        blocks[cur][-1] = (blocks[cur][-1], t)
    pos = {b: i for i, b in enumerate(order)}
    tot = {}
    for b in order:
        ins = blocks[b]
        if len(ins) < mn:
            continue
        c = {}
        for op, _ in ins:
            k = classify(op)
            c[k] = c.get(k, 0) + 1
            tot[k] = tot.get(k, 0) + 1
        back = ""
        for op, t in ins[-3:]:
            m = re.match(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", t)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in pos and pos[tgt] <= pos[b]:
                    back = f" loop->{tgt}"
        print(f"{b:16s} n={len(ins):5d} " + " ".join(f"{k}={c[k]}" for k in sorted(c)) + back)
    print("total", sum(tot.values()), " ".join(f"{k}={tot[k]}" for k in sorted(tot)))


if __name__ == "__main__":
    main()
