"""In-order issue model of a kernel's tile loop (one wave per SIMD), refined with the LDS queue:
DS ops complete in order, each occupying the CU's LDS pipe for its service time (x SHARE for the
co-resident waves of the CU), at most 15 outstanding (lgkmcnt is 4 bits: a 16th DS op stalls
issue); s_waitcnt lgkmcnt(k) waits for the (k+1)-th youngest to complete; MFMA pipe 32/16 cycles,
an MFMA holds issue 8 cycles; VALU 4 (transcendental / f64 8); ds_write2_b64 13 cycles of issue.
usage: python sim2.py <file.s> <kernel-substring> [SHARE] [BASE]"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
import estimate as e  # noqa: E402

SERVICE = {"ds_read_b32": 2, "ds_read_b64": 2, "ds_read_b64_tr_b16": 2, "ds_read_b128": 4, "ds_read2_b32": 4,
           "ds_read2_b64": 8, "ds_write_b32": 2, "ds_write_b64": 4, "ds_write2_b32": 4, "ds_write2_b64": 8,
           "ds_write_b128": 8, "ds_write2st64_b32": 4, "ds_bpermute_b32": 2}
ISSUE = {"ds_write_b32": 4, "ds_write_b64": 6, "ds_write2_b32": 6, "ds_write2_b64": 13, "ds_write_b128": 13,
         "ds_write2st64_b32": 6}


def run(path, sub, share=2.0, base=64):
    lines = [l for l in e.loop_body(path, sub) if l and not l.startswith(".")]
    t = pipe = 0.0
    ds_done = []  # completion times of issued DS ops, in order
    for ins in lines:
        op = ins.split()[0]
        if op.startswith("v_mfma"):
            t = max(t, pipe)
            pipe = t + (32 if "32x32" in op else 16)
            t += 8
        elif op == "s_nop":
            t += int(ins.split()[1]) + 1
        elif op == "s_waitcnt":
            m = re.search(r"lgkmcnt\((\d+)\)", ins)
            if m:
                k = int(m.group(1))
                if len(ds_done) > k:
                    t = max(t, ds_done[-k - 1])
        elif op.startswith("ds_"):
            if len(ds_done) >= 15:
                t = max(t, ds_done[-15])
            prev = ds_done[-1] if ds_done else 0.0
            svc = SERVICE.get(op, 4) * share
            done = max(t + base, prev + svc)
            ds_done.append(done)
            t += ISSUE.get(op, 4)
        elif op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")) or "_f64" in op:
            t += 8
        elif op.startswith("s_"):
            t += 1
        else:
            t += 4
    return max(t, pipe)


if __name__ == "__main__":
    share = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
    base = float(sys.argv[4]) if len(sys.argv) > 4 else 64
    print(f"{sys.argv[1]} {sys.argv[2]} cycles {run(sys.argv[1], sys.argv[2], share, base):.0f}")
