"""Loops of one kernel in an llvm-objdump -d listing of a gfx950 code object (A/B aid: no GPU).

usage: python tools/dis_loops.py LISTING.s KERNEL_SUBSTRING [--print START-END]
Lists every backward branch (a loop: its target .. the branch) with the instruction counts by class
in that address range; --print dumps the instructions of a range (hex addresses)."""
import re
import sys
from collections import Counter


def body(lines, sub):
    for i, l in enumerate(lines):
        if l.endswith(">:") and sub in l:
            j = i + 1
            while j < len(lines) and not lines[j].endswith(">:"):
                j += 1
            return l, lines[i + 1:j]
    raise SystemExit(f"no kernel matching {sub!r}")


def cls(op):
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sleep")):
        return "sync"
    for p, c in (("v_", "valu"), ("s_", "salu"), ("ds_", "lds"), ("global_", "vmem"), ("buffer_", "vmem"),
                 ("flat_", "vmem"), ("scratch_", "scratch")):
        if op.startswith(p):
            return c
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    name, b = body(lines, sub)
    base = int(name.split()[0], 16)
    ins = []
    for l in b:
        m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", l)
        if m:
            ins.append((int(m.group(3), 16) - base, m.group(1), m.group(2) + " " + l.split("//")[1]))
    if "--print" in sys.argv:
        a, z = (int(x, 16) for x in sys.argv[sys.argv.index("--print") + 1].split("-"))
        for ad, op, rest in ins:
            if a <= ad <= z:
                print(f"{ad:x}: {op} {rest}")
        return
    print(name, len(ins), "instructions", dict(Counter(cls(op) for _, op, _ in ins)))
    for ad, op, rest in ins:
        if op.startswith(("s_cbranch", "s_branch")):
            m = re.search(r"<[^+>]*\+0x([0-9a-f]+)>", rest)
            t = int(m.group(1), 16) if m else None
            if t is not None and t < ad:
                c = Counter(cls(o) for a2, o, _ in ins if t <= a2 <= ad)
                print(f"loop {t:x}..{ad:x}: {dict(c)}")


main()
