#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc --save-temps .s file, per basic
block (static counts), to see where a kernel's VALU issue slots go.

  python tools/isa_mix.py FILE.s KERNEL_SUBSTRING [--blocks]
"""
import collections
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    show_blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(name) + r"\w*:", l))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    total = collections.Counter()
    blocks = []
    cur, cnt = "entry", collections.Counter()
    for l in lines[start:end + 1]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append((cur, cnt))
            cur, cnt = m.group(1) + l[m.end():], collections.Counter()
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        cnt[op] += 1
        total[op] += 1
    blocks.append((cur, cnt))
    valu = sum(v for k, v in total.items() if k.startswith("v_"))
    print(f"kernel {name}: {sum(total.values())} instructions, {valu} VALU (static)")
    for k, v in total.most_common(40):
        print(f"  {k:28s} {v}")
    if show_blocks:
        for b, c in blocks:
            n = sum(c.values())
            if n > int(__import__("os").environ.get("ISA_MIN", "200")):
                vv = sum(v for k, v in c.items() if k.startswith("v_"))
                print(f"{b[:70]:70s} {n:6d} instr, {vv} valu; top: " +
                      ", ".join(f"{k}:{v}" for k, v in c.most_common(8)))


if __name__ == "__main__":
    main()
