"""Build-time ISA check of the split-precision train kernel's in-gap LDS reads (csrc/mlp_train.hip
X3_MACC6_RD).

Those inline-asm blocks issue six ds_read_b64_tr_b16 between their MFMAs and hand the
destination registers to the compiler as if the data were ready; the next block waits with
"s_waitcnt lgkmcnt(0)" before its MFMAs read them.  That is correct only if the register
allocator leaves those VGPRs untouched until that wait: a v_mov copy, a spill or a
rematerialisation in between would read (or clobber) registers whose LDS data is still in
flight and silently corrupt the weight gradients.  This script checks the invariant on the
code object actually built: for every in-gap ds_read_b64_tr_b16 (the asm blocks' runs of six
(AGPR-accumulating MFMA, read) pairs; the compiler's own reads are waited for by its own
counters), no instruction
may read or write any of its destination VGPRs before the next s_waitcnt lgkmcnt(0), and no
branch or label may intervene.

usage: python tools/check_asm_rd.py [libmhppo.so]   (exit 1 on a violation)"""
import os
import re
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
KERNEL = "k_mlp_train_x3"


def code_objects(path):
    """The gfx950 code objects of every clang offload bundle embedded in a host binary."""
    d = open(path, "rb").read()
    i = 0
    while True:
        i = d.find(MAGIC, i)
        if i < 0:
            return
        n = struct.unpack_from("<Q", d, i + 24)[0]
        p = i + 32
        for _ in range(n):
            off, size, ts = struct.unpack_from("<QQQ", d, p)
            p += 24
            triple = d[p:p + ts].decode()
            p += ts
            if "gfx950" in triple and size:
                yield d[i + off:i + off + size]
        i += len(MAGIC)


def regs(tok):
    """VGPR numbers named by one operand token (v7, v[4:5])."""
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def parse(line):
    """(mnemonic, [operand tokens]) of one objdump instruction line, or None."""
    t = line.split("//")[0].strip()
    if not t or t.endswith(":") or t.startswith("<"):
        return None
    op, _, rest = t.partition(" ")
    return op, [o.strip() for o in rest.split(",") if o.strip()]


def check_function(name, lines):
    """Violations in one kernel's disassembly (list of strings)."""
    bad, n_reads = [], 0
    insts = [(ln, p) for ln, p in ((ln, parse(ln)) for ln in lines)]
    ops = [(i, p) for i, (ln, p) in enumerate(insts) if p]

    def agpr_mfma(p):
        return p[0].startswith("v_mfma") and p[1][0].startswith("a[")

    # The asm blocks are runs of six (MFMA accumulating in AGPRs, ds_read_b64_tr_b16) pairs.  The
    # compiler's own MFMAs in this translation unit write VGPRs (-amdgpu-mfma-vgpr-form) and its
    # own LDS reads are covered by its own counted waits.
    asm_reads = set()
    for n in range(len(ops) - 11):
        if all(agpr_mfma(ops[n + 2 * q][1]) and ops[n + 2 * q + 1][1][0] == "ds_read_b64_tr_b16" for q in range(6)):
            asm_reads.update(ops[n + 2 * q + 1][0] for q in range(6))
    for k, (ln, pi) in enumerate(insts):
        if k not in asm_reads:
            continue
        n_reads += 1
        pending = regs(pi[1][0])
        for ln2, p2 in insts[k + 1:]:
            if p2 is None:
                if ln2.strip().endswith(":"):
                    bad.append(f"{name}: label before the wait for {pi[1][0]} ({ln.strip()})")
                    break
                continue
            op2, ops2 = p2
            if op2 == "s_waitcnt" and "lgkmcnt(0)" in " ".join(ops2):
                break
            if op2.startswith(("s_branch", "s_cbranch", "s_setpc", "s_endpgm")):
                bad.append(f"{name}: branch before the wait for {pi[1][0]} ({ln.strip()})")
                break
            used = set().union(*[regs(o) for o in ops2]) if ops2 else set()
            if op2 == "ds_read_b64_tr_b16":  # a later in-gap read: only its address may not overlap
                used = set().union(*[regs(o) for o in ops2[1:]]) if len(ops2) > 1 else set()
                if regs(ops2[0]) & pending:
                    bad.append(f"{name}: {ln2.strip()} overwrites in-flight {pi[1][0]}")
                    break
            if used & pending:
                bad.append(f"{name}: '{ln2.strip()}' touches in-flight {pi[1][0]} of '{ln.strip()}'")
                break
    # The hand-placed backward's one-MFMA asm statements (mac1 / mac1_16: AGPR accumulator, no
    # s_nop inside) rely on their A / B operands never being written by a VALU instruction in the
    # two wait states before them (VALU write -> MFMA SrcA/B/C read: 2 wait states on gfx950; hipcc
    # pads nothing around an asm statement).  Every AGPR-accumulating MFMA is checked: walking back
    # over the instructions before it, counting one wait state per instruction and N + 1 per
    # s_nop N, no v_* instruction within 2 wait states may write a VGPR / AGPR it reads as A, B or C
    # (a v_accvgpr_mov / _write of an accumulator the compiler moved between registers).
    def dst_regs(ops_):
        t = ops_[0] if ops_ else ""
        m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", t)
        if m:
            return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        m = re.fullmatch(r"([va])(\d+)", t)
        return {(m.group(1), int(m.group(2)))} if m else set()
    for n, (i, p) in enumerate(ops):
        if not agpr_mfma(p):
            continue
        srcs = set()
        for tok in p[1][1:4]:  # A, B and C (an accumulator a compiler copy / write just set up)
            m = re.fullmatch(r"([va])\[(\d+):(\d+)\]", tok)
            if m:
                srcs |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        states, k = 0, n - 1
        while k >= 0 and states < 2:
            j, q = ops[k]
            if any(insts[x][0].strip().endswith(":") for x in range(j + 1, i)):
                break  # a label in between: another block's tail, not this straight-line run
            if q[0] == "s_nop":
                states += int(q[1][0], 0) + 1
            else:
                if q[0].startswith("v_") and not q[0].startswith("v_mfma") and dst_regs(q[1]) & srcs:
                    bad.append(f"{name}: '{insts[j][0].strip()}' writes an operand of '{insts[i][0].strip()}' "
                               f"{states} wait states before it")
                states += 1
            k -= 1
    return bad, n_reads


def main(path):
    total_reads, bad, nfun = 0, [], 0
    for co in code_objects(path):
        tmp = "/tmp/mhppo_check_asm_rd.co"
        with open(tmp, "wb") as f:
            f.write(co)
        dis = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", tmp], capture_output=True, text=True,
                             check=True).stdout
        os.unlink(tmp)
        if KERNEL not in dis:
            continue
        funcs = re.split(r"\n(?=[0-9a-f]+ <)", dis)
        for fn in funcs:
            head = fn.split("\n", 1)[0]
            if KERNEL not in head:
                continue
            nfun += 1
            b, n = check_function(head.strip(), fn.split("\n")[1:])
            bad += b
            total_reads += n
    if nfun == 0:
        print(f"check_asm_rd: no {KERNEL} kernel in {path}")
        return 1
    if total_reads == 0:
        print("check_asm_rd: found no in-gap reads (did the asm blocks change?)")
        return 1
    for b in bad:
        print("VIOLATION", b)
    print(f"check_asm_rd: {nfun} kernels, {total_reads} in-gap ds_read_b64_tr_b16, {len(bad)} violations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "mh-ppo_amd", "mhppo", "lib",
                                                                        "libmhppo.so")))
