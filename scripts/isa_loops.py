"""Instruction mix per basic block of one kernel in a device assembly file
(``hipcc --cuda-device-only -S``): finds the kernel by a name substring and
prints, for every block ending in a backward branch (a loop) and for the
whole kernel, the counts of MFMA / VALU / SALU / LDS / VMEM / waitcnt
instructions.

    python scripts/isa_loops.py build/isa/conv_h3.s conv_h3r_kernelILi7ELi4ELi9ELi600ELi2ELb0ELb0E
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("ds_",)):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_load", "s_buffer")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines)
                 if l.startswith("_Z") and name in l.split(":")[0] and ":" in l)
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = Counter()
    order = [cur]
    ops = Counter()
    back = {}
    for l in lines[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end") or s.startswith("s_endpgm"):
            if s.startswith("s_endpgm"):
                blocks[cur]["salu"] += 1
            break
        if re.match(r"^\.LBB\d+_\d+:", s):
            cur = s.split(":")[0]
            blocks[cur] = Counter()
            order.append(cur)
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        c = classify(op)
        blocks[cur][c] += 1
        ops[c] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = s.split()[-1]
            if tgt in blocks and tgt != "entry":
                back[cur] = tgt
    print("kernel total:", dict(ops))
    for b in order:
        if b in back:
            # the loop = blocks from its target to this block
            i0, i1 = order.index(back[b]), order.index(b)
            tot = Counter()
            for x in order[i0:i1 + 1]:
                tot.update(blocks[x])
            m = tot["mfma"] or 1
            print("loop %s..%s: %s  valu/mfma %.2f salu/mfma %.2f" % (
                back[b], b, dict(tot), tot["valu"] / m, tot["salu"] / m))


if __name__ == "__main__":
    main()
