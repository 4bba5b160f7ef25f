"""Per-kernel summary (calls, total/avg/min/max ns, % of GPU time) from a rocprofv3
rocpd database (run_results.db) — same columns as rocprofv3's kernel_stats.csv."""
import sqlite3
import sys


def main(db, out=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                     "from kernels group by name order by sum(end-start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    lines = ['"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"']
    for n, k, s, a, mn, mx in rows:
        lines.append(f'"{n}",{k},{s},{a:.1f},{100.0 * s / tot:.3f},{mn},{mx}')
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    return text


if __name__ == "__main__":
    print(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None))
