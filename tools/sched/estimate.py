"""Estimate what re-ordering alone could gain on a kernel's tile loop: per region (straight-line
run between branches / labels / vmcnt waits), an in-order issue model vs a critical-path list
schedule over the register/LDS dependency DAG (same latency and issue model).
usage: python tools/sched/estimate.py <file.s> <kernel-substring>"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa import defs_uses, issue_cost, mfma_pipe  # noqa: E402


def loop_body(path, sub):
    s = open(path).read()
    m = re.search(r"^(\S*" + re.escape(sub) + r"\S*):", s, re.M)
    body = s[m.start():s.index(".Lfunc_end", m.start())].split("\n")
    st = [n for n, l in enumerate(body) if "Loop Header: Depth=1" in l][0]
    labels = {}
    for n, ln in enumerate(body):
        mm = re.match(r"^(\.LBB\w+):", ln.strip())
        if mm:
            labels[mm.group(1)] = n
    end = st
    for n, ln in enumerate(body):
        mm = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", ln)
        if mm and labels.get(mm.group(1) or mm.group(2)) == st:
            end = max(end, n)
    return [l.split(";")[0].strip() for l in body[st:end + 1]]


def regions(lines):
    cur = []
    for l in lines:
        if not l:
            continue
        if l.startswith(".LBB") or l.startswith("."):
            if cur:
                yield cur
            cur = []
            continue
        op = l.split()[0]
        if op.startswith(("s_cbranch", "s_branch")) or (op == "s_waitcnt" and "vmcnt" in l):
            if cur:
                yield cur
            cur = []
            continue
        cur.append(l)
    if cur:
        yield cur


def lat(p, c, reg):
    op, cls = p["op"], p["cls"]
    if cls == "mfma":
        if c["cls"] == "mfma" and reg in c.get("srcc", ()):
            return mfma_pipe(op)
        return 2 * mfma_pipe(op) + 4
    if cls == "ds":
        return 120
    if cls == "vmem":
        return 500
    if cls == "salu":
        return 2
    if op.endswith("_f64") or op.startswith(("v_exp", "v_log", "v_rcp", "v_sqrt", "v_rsq")):
        return 16
    return 8


def build(reg_lines):
    ins = []
    for l in reg_lines:
        op, cls, d, u = defs_uses(l)
        if cls in ("wait", "nop"):
            continue
        it = {"txt": l, "op": op, "cls": cls, "d": d, "u": u, "cost": issue_cost(op, cls)}
        if cls == "mfma":
            toks = [t.strip() for t in l.split(None, 1)[1].split(",")]
            from isa import regs
            it["srcc"] = set(regs(toks[3])) if len(toks) > 3 else set()
        ins.append(it)
    n = len(ins)
    preds = [dict() for _ in range(n)]
    last_def, last_uses = {}, {}
    last_dsw, dsr_since = None, []
    for i, it in enumerate(ins):
        for r in it["u"]:
            if r in last_def:
                j = last_def[r]
                preds[i][j] = max(preds[i].get(j, 0), lat(ins[j], it, r))
        for r in it["d"]:
            for j in last_uses.get(r, []):
                if j != i:
                    preds[i][j] = max(preds[i].get(j, 0), 1)
            if r in last_def:
                j = last_def[r]
                preds[i][j] = max(preds[i].get(j, 0), 1)
        if it["cls"] == "ds":
            w = it["op"].startswith(("ds_write", "ds_store"))
            if last_dsw is not None:
                preds[i][last_dsw] = max(preds[i].get(last_dsw, 0), 1)
            if w:
                for j in dsr_since:
                    preds[i][j] = max(preds[i].get(j, 0), 1)
                last_dsw, dsr_since = i, []
            else:
                dsr_since.append(i)
        for r in it["u"]:
            last_uses.setdefault(r, []).append(i)
        for r in it["d"]:
            last_def[r] = i
            last_uses[r] = []
    return ins, preds


def inorder(ins, preds):
    t = pipe = 0
    done = {}
    for i, it in enumerate(ins):
        ready = max([done[j] + l for j, l in preds[i].items()] + [0])
        t = max(t, ready)
        if it["cls"] == "mfma":
            t = max(t, pipe)
            pipe = t + mfma_pipe(it["op"])
        done[i] = t
        t += it["cost"]
    return max(t, pipe)


def listsched(ins, preds):
    n = len(ins)
    succ = [[] for _ in range(n)]
    for i in range(n):
        for j, l in preds[i].items():
            succ[j].append((i, l))
    prio = [0] * n
    for i in reversed(range(n)):
        prio[i] = ins[i]["cost"] + max([l + prio[k] for k, l in succ[i]] + [0])
    npred = [len(p) for p in preds]
    earliest = [0] * n
    ready = [i for i in range(n) if npred[i] == 0]
    t = pipe = 0
    left = n
    order = []
    while left:
        cand = [i for i in ready if earliest[i] <= t and (ins[i]["cls"] != "mfma" or pipe <= t)]
        if not cand:
            nxt = [earliest[i] for i in ready if earliest[i] > t]
            nxt += [pipe] if any(ins[i]["cls"] == "mfma" for i in ready) and pipe > t else []
            t = min(nxt) if nxt else t + 1
            continue
        i = max(cand, key=lambda k: (prio[k], -k))
        ready.remove(i)
        order.append(i)
        if ins[i]["cls"] == "mfma":
            pipe = t + mfma_pipe(ins[i]["op"])
        start = t
        t += ins[i]["cost"]
        left -= 1
        for k, l in succ[i]:
            earliest[k] = max(earliest[k], start + l)
            npred[k] -= 1
            if npred[k] == 0:
                ready.append(k)
    return max(t, pipe), order


def main(path, sub):
    tot_in = tot_ls = tot_issue = tot_pipe = 0
    for reg in regions(loop_body(path, sub)):
        ins, preds = build(reg)
        if not ins:
            continue
        a = inorder(ins, preds)
        b, _ = listsched(ins, preds)
        iss = sum(x["cost"] for x in ins)
        pp = sum(mfma_pipe(x["op"]) for x in ins if x["cls"] == "mfma")
        tot_in += a
        tot_ls += b
        tot_issue += iss
        tot_pipe += pp
        if len(ins) > 40:
            print(f"region {len(ins):5d} instrs: in-order {a:6d}  list {b:6d}  issue {iss:6d}  mfma-pipe {pp:6d}")
    print(f"TOTAL in-order {tot_in}  list {tot_ls}  issue {tot_issue}  mfma-pipe {tot_pipe}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])


def dual(path, sub):
    """Two independent copies of every region list-scheduled together (upper bound for two
    tiles in flight per wave, registers unlimited)."""
    tot = tot1 = 0
    for reg in regions(loop_body(path, sub)):
        ins, preds = build(reg)
        if not ins:
            continue
        n = len(ins)
        ins2 = ins + [dict(x) for x in ins]
        preds2 = preds + [{j + n: l for j, l in p.items()} for p in preds]
        b, _ = listsched(ins2, preds2)
        tot += b
        tot1 += listsched(ins, preds)[0]
    print(f"two tiles: list {tot} = {tot / 2:.0f} per tile (one tile: {tot1})")


def stalls(path, sub, top=25):
    """Where the in-order model waits: the instructions whose issue is delayed most (by a
    dependency or the MFMA pipe), with their region index and position."""
    res = []
    for ri, reg in enumerate(regions(loop_body(path, sub))):
        ins, preds = build(reg)
        t = pipe = 0
        done = {}
        for i, it in enumerate(ins):
            ready = max([done[j] + l for j, l in preds[i].items()] + [0])
            t0 = t
            t = max(t, ready)
            why = "dep"
            if it["cls"] == "mfma" and pipe > t:
                t, why = pipe, "pipe"
            if it["cls"] == "mfma":
                pipe = t + mfma_pipe(it["op"])
            if t > t0:
                src = max(preds[i].items(), key=lambda x: done[x[0]] + x[1])[0] if preds[i] else None
                res.append((t - t0, ri, i, why, it["txt"][:60], ins[src]["txt"][:50] if src is not None else ""))
            done[i] = t
            t += it["cost"]
    res.sort(reverse=True)
    agg = {}
    for w, ri, i, why, a, b in res:
        k = (why, a.split()[0], b.split()[0] if b else "")
        agg[k] = agg.get(k, 0) + w
    for k, v in sorted(agg.items(), key=lambda x: -x[1])[:top]:
        print(f"{v:6d}  {k}")
