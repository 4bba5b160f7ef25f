"""Instruction histogram of a kernel's longest loop in a hipcc -S listing (A/B tool).
Usage: python tools/asm_loop.py <file.s> <kernel-name-substring> [top]"""
import collections
import re
import sys


def main(path, sub, top=30):
    s = open(path).read()
    m = re.search(r"^(\S*" + re.escape(sub) + r"\S*):", s, re.M)
    i = m.start()
    body = s[i:s.index(".Lfunc_end", i)].split("\n")
    labels = {}
    for n, ln in enumerate(body):
        mm = re.match(r"^(\.LBB\w+):", ln.strip())
        if mm:
            labels[mm.group(1)] = n
    loops = []
    for n, ln in enumerate(body):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if mm:
            t = mm.group(1) or mm.group(2)
            if t in labels and labels[t] < n:
                loops.append((labels[t], n))
    outer = [lp for lp in loops if "Loop Header: Depth=1" in body[lp[0]]]  # the tile loop, not
    a, b = max(outer or loops, key=lambda x: x[1] - x[0])                 # structurizer back-jumps
    c = collections.Counter()
    for ln in body[a:b]:
        t = ln.strip().split(" ")[0]
        if t and not t.startswith((".", ";")) and not t.endswith(":"):
            c[t] += 1
    print(m.group(1), "loop instructions", sum(c.values()))
    for k, v in sorted(c.items(), key=lambda x: -x[1])[:top]:
        print(f"{v:5d} {k}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30)
