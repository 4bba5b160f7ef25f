"""List the VGPRs a kernel's main loop reads but never writes (loop invariants held in
registers) in a hipcc -S listing.  Usage: python tools/asm_invariants.py <file.s> <kernel-substring>"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return [int(m.group(1))] if m else []


def main(path, sub):
    s = open(path).read()
    m = re.search(r"^(\S*" + re.escape(sub) + r"\S*):", s, re.M)
    body = s[m.start():s.index(".Lfunc_end", m.start())].split("\n")
    hdr = [n for n, ln in enumerate(body) if "Loop Header: Depth=1" in ln][-1]
    lab = body[hdr].split(":")[0]
    end = max(n for n, ln in enumerate(body) if re.search(r"s_c?branch\w*\s+" + re.escape(lab) + r"\b", ln))
    written, read = set(), {}
    for ln in body[hdr:end]:
        t = ln.strip()
        if not t or t.startswith((";", ".")):
            continue
        op, _, rest = t.partition(" ")
        ops = [o.strip() for o in rest.split(";")[0].split(",")]
        stores = op.startswith(("ds_write", "scratch_store", "global_store", "buffer_store")) or op.startswith("v_cmp")
        for i, o in enumerate(ops):
            for r in regs(o):
                if i == 0 and not stores:
                    written.add(r)
                else:
                    read.setdefault(r, t[:70])
    inv = sorted(r for r in read if r not in written)
    print(f"{len(inv)} loop-invariant VGPRs")
    for r in inv:
        print(f"v{r}: {read[r]}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
