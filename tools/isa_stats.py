"""Static instruction mix of one kernel in a `hipcc --cuda-device-only -S` listing (A/B aid: no GPU).

usage: python tools/isa_stats.py FILE.s KERNEL_SUBSTRING [--loops]
Prints the kernel's VGPR / SGPR / LDS / scratch figures and its instruction counts by class
(v_, s_, ds_, global_/buffer_, branches); with --loops, the same per basic block that ends in a
backward branch (the loop bodies), which is what the PMC instruction counts scale with."""
import re
import sys
from collections import Counter


def kernel_body(text: str, sub: str):
    names = [m.group(1) for m in re.finditer(r"^(\S+):\s*;\s*@\1\s*$", text, re.M) if sub in m.group(1)]
    if not names:
        names = [m.group(1) for m in re.finditer(r"^(_Z\S+):", text, re.M) if sub in m.group(1)]
    if not names:
        raise SystemExit(f"no kernel matching {sub!r}")
    name = names[0]
    start = text.index(f"\n{name}:") + 1
    end = text.index(".Lfunc_end", start)
    meta = {}
    for key, pat in (("vgpr", r"; NumVgprs: (\d+)"), ("agpr", r"; NumAgprs: (\d+)"), ("sgpr", r"; NumSgprs: (\d+)"),
                     ("scratch", r"; ScratchSize: (\d+)"), ("occupancy", r"; Occupancy: (\d+)"),
                     ("lds", r"; LDSByteSize: (\d+)")):
        m = re.search(pat, text[end:end + 20000])
        if m:
            meta[key] = int(m.group(1))
    return name, text[start:end], meta


def classify(ins: str) -> str:
    if ins.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if ins.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_setprio", "s_sleep")):
        return "sync"
    if ins.startswith("v_"):
        return "valu"
    if ins.startswith("s_"):
        return "salu"
    if ins.startswith("ds_"):
        return "lds"
    if ins.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    text = open(path).read()
    name, body, meta = kernel_body(text, sub)
    print(name, meta)
    lines = [l.strip() for l in body.splitlines()]
    tot = Counter()
    blocks, cur, label = [], Counter(), "entry"
    for l in lines:
        if re.match(r"^\.LBB\S+:", l):
            blocks.append((label, cur))
            cur, label = Counter(), l.split(":")[0]
            continue
        if not l or l.startswith((";", ".")):
            continue
        ins = l.split()[0]
        k = classify(ins)
        tot[k] += 1
        cur[k] += 1
        if ins.startswith("s_cbranch") or ins.startswith("s_branch"):
            tgt = l.split()[-1]
            cur["->" + tgt] += 1
    blocks.append((label, cur))
    print("total", dict(tot))
    if "--loops" in sys.argv:
        order = [b[0] for b in blocks]
        for i, (lab, c) in enumerate(blocks):
            back = [k[2:] for k in c if k.startswith("->") and k[2:] in order and order.index(k[2:]) <= i]
            for b in back:  # the loop = blocks from the target to this latch (layout order)
                j = order.index(b)
                loop = Counter()
                for _, cc in blocks[j:i + 1]:
                    loop.update({k: v for k, v in cc.items() if not k.startswith("->")})
                print(f"loop {b} .. {lab} ({i - j + 1} blocks): " + ", ".join(f"{k}={v}" for k, v in sorted(loop.items())))


if __name__ == "__main__":
    main()
