"""Minimal gfx950 asm parser for the post-RA study tools: instruction -> (defs, uses, class).
Register sets are expanded to unit names (v12, a3, s40, vcc_lo/hi as 'vcc', 'scc', 'exec', 'm0')."""
import re

_RANGE = re.compile(r"^([vas])\[(\d+):(\d+)\]$")
_ONE = re.compile(r"^([vas])(\d+)$")


def regs(tok):
    tok = tok.strip().rstrip(",")
    if tok.startswith("-"):
        tok = tok[1:]
    m = _RANGE.match(tok)
    if m:
        return [f"{m.group(1)}{i}" for i in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = _ONE.match(tok)
    if m:
        return [tok]
    if tok in ("vcc", "vcc_lo", "vcc_hi"):
        return ["vcc"]
    if tok in ("exec", "exec_lo", "exec_hi"):
        return ["exec"]
    if tok == "m0":
        return ["m0"]
    if tok in ("scc",):
        return ["scc"]
    return []


def split_ops(ins):
    parts = ins.split(None, 1)
    op = parts[0]
    rest = parts[1] if len(parts) > 1 else ""
    # drop modifiers (offset:, offen, etc.), keep operand list
    toks = [t.strip() for t in rest.split(",")]
    ops = []
    for t in toks:
        t = t.split()[0] if t else t
        ops.append(t)
    return op, ops


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op in ("s_waitcnt",):
        return "wait"
    if op == "s_nop":
        return "nop"
    if op.startswith(("s_cbranch", "s_branch", "s_barrier", "s_setprio", "s_sleep", "s_endpgm")):
        return "ctrl"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def defs_uses(ins):
    op, ops = split_ops(ins)
    cls = classify(op)
    d, u = [], []
    if cls in ("wait", "nop", "ctrl"):
        if op.startswith("s_cbranch_scc"):
            u.append("scc")
        if op.startswith("s_cbranch_vcc"):
            u.append("vcc")
        if op.startswith("s_cbranch_exec"):
            u.append("exec")
        return op, cls, d, u
    if cls == "ds":
        if op.startswith(("ds_write", "ds_store")):
            for t in ops:
                u += regs(t)
        else:
            d += regs(ops[0])
            for t in ops[1:]:
                u += regs(t)
        u.append("exec")
        return op, cls, d, u
    if cls == "vmem":
        lds = " lds" in ins
        if op.startswith(("buffer_store", "global_store")) or lds:
            for t in ops:
                u += regs(t)
            if lds:
                u.append("m0")
        else:
            d += regs(ops[0])
            for t in ops[1:]:
                u += regs(t)
        u.append("exec")
        return op, cls, d, u
    if cls == "salu":
        if op.startswith(("s_cmp", "s_bitcmp")):
            d.append("scc")
            for t in ops:
                u += regs(t)
            return op, cls, d, u
        d += regs(ops[0])
        for t in ops[1:]:
            u += regs(t)
        if op.startswith(("s_addc", "s_subb", "s_cselect", "s_cmov")):
            u.append("scc")
        if not op.startswith(("s_mov", "s_movk", "s_getreg", "s_setreg")):
            d.append("scc")
        if "saveexec" in op:
            d.append("exec")
            u.append("exec")
        return op, cls, d, u
    if cls in ("valu", "mfma"):
        if op.startswith("v_cmp") and op.endswith("_e32"):
            d.append("vcc")
            for t in ops:
                u += regs(t)
        elif op.startswith("v_cmpx"):
            d.append("exec")
            for t in ops:
                u += regs(t)
        else:
            d += regs(ops[0])
            rest = ops[1:]
            # VOP3 carry-out forms: v_add_co_u32_e64 v, s[..], a, b
            if ("_co_" in op or op.startswith(("v_addc", "v_subb"))) and op.endswith("_e64"):
                d += regs(rest[0])
                rest = rest[1:]
            for t in rest:
                u += regs(t)
            if op.endswith("_e32") and ("_co_" in op or op.startswith(("v_addc", "v_subb"))):
                d.append("vcc")
            if op.startswith(("v_cndmask_b32_e32", "v_addc", "v_subb")) and op.endswith("_e32"):
                u.append("vcc")
        u.append("exec")
        return op, cls, d, u
    return op, cls, d, u


def issue_cost(op, cls):
    if cls == "mfma":
        return 8
    if cls == "nop":
        return 0
    if cls in ("salu", "wait", "ctrl", "smem"):
        return 1
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return 8
    if op.endswith("_f64") or "_f64_" in op:
        return 8
    return 4


def mfma_pipe(op):
    if "32x32x16" in op or "32x32x2" in op:
        return 32
    return 16
