"""Per-kernel HBM traffic per launch from rocprofv3 PMC passes (separate FETCH_SIZE and
WRITE_SIZE runs, counter_collection.csv), with the gfx950 correction of
MI355X_MICROARCH.md §HBM: FETCH_SIZE counts half the bytes of wide streaming reads
(it is TCC_EA0_RDREQ x 64 B), so reads = 2 x FETCH_SIZE; WRITE_SIZE is exact.
FETCH_SIZE / WRITE_SIZE are reported in KiB.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _collect(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            per[name].append(float(row["Counter_Value"]))
    return per


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("(anonymous namespace)::", "")


def main(fetch_dir, write_dir, out):
    fe = _collect(fetch_dir, "FETCH_SIZE")
    wr = _collect(write_dir, "WRITE_SIZE")
    res = {}
    for name in sorted(set(fe) | set(wr)):
        f = fe.get(name, [])
        w = wr.get(name, [])
        fk = sum(f) / len(f) if f else None
        wk = sum(w) / len(w) if w else None
        res[short(name) + ("" if short(name) == name else "") + f" [{name[:160]}]"] = {
            "launches_fetch": len(f), "launches_write": len(w),
            "fetch_kib_raw": fk, "write_kib": wk,
            "read_bytes_corrected": None if fk is None else 2.0 * fk * 1024.0,
            "write_bytes": None if wk is None else wk * 1024.0,
            "hbm_bytes_per_launch": None if (fk is None or wk is None) else 2.0 * fk * 1024.0 + wk * 1024.0,
        }
    json.dump({"correction": "reads = 2 x FETCH_SIZE (gfx950), FETCH_SIZE/WRITE_SIZE in KiB", "kernels": res},
              open(out, "w"), indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -(kv[1]["hbm_bytes_per_launch"] or 0))[:15]:
        print(f"{k[:90]:90s} {v['hbm_bytes_per_launch']}")


if __name__ == "__main__":
    main(*sys.argv[1:4])
