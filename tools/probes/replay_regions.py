"""Micro-probe generator (tools only): replay a range of the train kernel's scheduling regions
(the instruction text between sched_barriers of its main tile loop, from `hipcc -S`) as one
inline-asm block in a standalone kernel, one wave per SIMD, and time it with s_memtime.

Variants rewrite the text to isolate what a block's time is made of:
  asis      the regions as compiled
  mfma      the MFMAs only (same operands, same order)
  nods      no LDS instructions / waits (VALU + MFMA)
  nowr      no LDS stores;  nord: no LDS loads / waits;  noval: no VALU but the address adds
  agpr      the VGPR accumulators of the on-chain MFMAs renamed into free AGPRs
  agpr_nods both
Every register starts at zero and the LDS instructions' addresses are checked on the host to stay
inside the 64 KiB the probe allocates (registers written by the replayed text are only allowed
as addresses when they are `v_add_u32 vX, imm, vY` of an unwritten register).

usage: python3 replay_regions.py <asm.s> <kernel-substring> <name>:<lo>-<hi> ... > probe.hip
build: hipcc --offload-arch=gfx950 -O3 -o probe probe.hip
"""
import re
import sys

LDS_BYTES = 65536
REPS = 8
KINDS = ("asis", "mfma", "nods", "nowr", "nord", "noval")


def regions(path, sub):
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
    outer = [lp for lp in loops if "Loop Header: Depth=1" in body[lp[0]]]
    a, b = max(outer or loops, key=lambda x: x[1] - x[0])
    reg, out = 0, {}
    for ln in body[a:b + 1]:
        if "sched_barrier" in ln:
            reg += 1
            continue
        t = ln.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        out.setdefault(reg, []).append(t.split(";")[0].rstrip())
    return out


def vregs(tok):
    """VGPR numbers named by one operand token (v5, v[2:17])."""
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return [int(m.group(1))]
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return []


def ops(ins):
    parts = ins.split(None, 1)
    if len(parts) == 1:
        return parts[0], []
    return parts[0], [x.strip() for x in re.split(r",(?![^\[]*\])", parts[1])]


def check_lds(lines):
    """Every ds_* address provably below LDS_BYTES with all registers starting at 0."""
    written, known = set(), {}
    for ins in lines:
        op, args = ops(ins)
        if op.startswith("ds_"):
            addr = args[1] if op.startswith("ds_read") or op.startswith("ds_bpermute") else args[0]
            if op.startswith("ds_write"):
                addr = args[0]
            r = vregs(addr.split()[0])[0]
            base = known.get(r, 0 if r not in written else None)
            if base is None:
                raise SystemExit(f"unsafe LDS address register v{r} in: {ins}")
            offs = [int(x) for x in re.findall(r"offset\d?:(\d+)", ins)] or [0]
            scale = 8 if "2_b64" in op else (4 if "2_b32" in op else 1)
            hi = base + max(offs) * scale + 16
            if hi > LDS_BYTES:
                raise SystemExit(f"LDS address {hi} past {LDS_BYTES}: {ins}")
        if args and not op.startswith("ds_write") and not op.startswith("s_") and not op.startswith("v_mfma"):
            dst = vregs(args[0])
            if op in ("v_add_u32_e32", "v_add3_u32") and len(dst) == 1:
                tot = 0
                for a in args[1:]:
                    if re.fullmatch(r"(0x[0-9a-f]+|\d+)", a):
                        tot += int(a, 0)
                    elif vregs(a) and (vregs(a)[0] not in written or vregs(a)[0] in known):
                        tot += known.get(vregs(a)[0], 0)
                    else:
                        tot = None
                        break
                if tot is not None:
                    known[dst[0]] = tot
                    written.add(dst[0])
                    continue
            for r in dst:
                written.add(r)
                known.pop(r, None)
        if op.startswith("v_mfma") and args[0].startswith("v"):
            for r in vregs(args[0]):
                written.add(r)
                known.pop(r, None)


def variant(lines, kind):
    out = []
    used_a = set()
    for ins in lines:
        for m in re.finditer(r"a\[(\d+):(\d+)\]|a(\d+)\b", ins):
            if m.group(3):
                used_a.add(int(m.group(3)))
            else:
                used_a.update(range(int(m.group(1)), int(m.group(2)) + 1))
    free = [a for a in range(256) if a not in used_a]
    ren = {}
    for ins in lines:
        op, args = ops(ins)
        is_ds = op.startswith("ds_") or op.startswith("s_waitcnt")
        if kind == "mfma" and not op.startswith("v_mfma"):
            continue
        if kind in ("nods", "agpr_nods") and is_ds:
            continue
        if kind == "nowr" and op.startswith("ds_write"):
            continue
        if kind == "nord" and (op.startswith("ds_read") or op.startswith("s_waitcnt")):
            continue
        if kind == "noval" and op.startswith("v_") and not op.startswith("v_mfma") and not op.startswith("v_add_u32"):
            continue
        if kind in ("agpr", "agpr_nods") and op.startswith("v_mfma") and args[0].startswith("v["):
            d = args[0]
            if d not in ren:
                n = len(vregs(d))
                fs = set(free)
                st = next((i for i in range(0, 256 - n + 1, 4) if all(j in fs for j in range(i, i + n))), None)
                if st is None:  # no room: keep this accumulator in VGPRs
                    out.append(ins)
                    continue
                ren[d] = f"a[{st}:{st + n - 1}]"
                free = [j for j in free if not st <= j < st + n]
            args = [ren[d] if a == d else a for a in args]
            ins = op + " " + ", ".join(args)
        out.append(ins)
    return out


def emit(blocks):
    print("// generated by tools/probes/replay_regions.py", file=sys.stdout)
    print("#include <hip/hip_runtime.h>\n#include <stdio.h>")
    clob = ", ".join([f'"v{i}"' for i in range(256)] + [f'"a{i}"' for i in range(256)] +
                     ['"vcc"', '"s40"', '"s41"', '"s42"', '"s43"', '"memory"'])
    init = "".join(f"v_mov_b32 v{i}, 0\\n" for i in range(256)) + \
           "".join(f"v_accvgpr_write_b32 a{i}, 0\\n" for i in range(256))
    names = []
    for name, kinds in blocks:
        for kind, lines in kinds:
            kn = f"{name}_{kind}"
            names.append((kn, sum(1 for x in lines if x.startswith("v_mfma")), len(lines)))
            body = "".join(x.replace('"', '\\"') + "\\n" for x in lines)
            print(f"__global__ void __launch_bounds__(256) k_{kn}(unsigned long long *cyc) {{")
            print("  extern __shared__ float lds[];")
            print("  unsigned long long t;")
            print(f'  asm volatile("{init}s_waitcnt lgkmcnt(0)\\n'
                  f's_memtime s[40:41]\\ns_waitcnt lgkmcnt(0)\\n"')
            for _ in range(REPS):
                print(f'               "{body}"')
            print('               "s_waitcnt lgkmcnt(0)\\ns_nop 15\\ns_nop 15\\ns_nop 15\\ns_nop 15\\n'
                  's_memtime s[42:43]\\ns_waitcnt lgkmcnt(0)\\n'
                  's_sub_u32 s42, s42, s40\\ns_subb_u32 s43, s43, s41\\ns_mov_b64 %0, s[42:43]\\n"')
            print(f'               : "=s"(t) : : {clob});')
            print("  if (threadIdx.x == 0) cyc[blockIdx.x] = t;")
            print("  (void)lds;\n}")
    print("int main() {\n  unsigned long long *cyc, h[256];\n  hipMalloc(&cyc, sizeof(h));")
    for kn, nm, ni in names:
        print(f"  hipFuncSetAttribute((const void *)k_{kn}, hipFuncAttributeMaxDynamicSharedMemorySize, {LDS_BYTES});")
        print("  for (int rep = 0; rep < 3; rep++)")
        print(f"    hipLaunchKernelGGL(k_{kn}, dim3(256), dim3(256), {LDS_BYTES}, 0, cyc);")
        print("  hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);")
        print("  { double s = 0; for (int i = 0; i < 256; i++) s += h[i];")
        print(f'    printf("%-22s %3d mfma %4d instr: %7.0f cycles per pass (%.1f per MFMA)\\n", "{kn}", {nm}, {ni},'
              f" (s / 256 - 64) / {REPS}, (s / 256 - 64) / {REPS} / {max(nm, 1)}); }}")
    print("  return 0;\n}")


def main():
    path, sub = sys.argv[1], sys.argv[2]
    regs = regions(path, sub)
    blocks = []
    for spec in sys.argv[3:]:
        name, rng = spec.split(":")
        lo, hi = [int(x) for x in rng.split("-")]
        # scalar sources of VALU address arithmetic (an LDS base in an SGPR) read as 0
        lines = [re.sub(r"(v_add3_u32 v\d+, )s\d+", r"\g<1>0", x) for r in range(lo, hi + 1) for x in regs.get(r, [])]
        if any(re.search(r"\bs\[|\bs\d+\b|exec|\.LBB|s_cbranch|s_branch", x) for x in lines):
            raise SystemExit(f"{name}: scalar registers / branches in the range")
        check_lds(lines)
        kinds = [(k, variant(lines, k)) for k in KINDS]
        blocks.append((name, kinds))
    emit(blocks)


if __name__ == "__main__":
    main()
