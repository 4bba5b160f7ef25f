"""Mean per-dispatch SQ counter values per kernel from rocprofv3 --pmc directories.
usage: python tools/pmc_sq.py [--kernel SUBSTR] <dir> [<dir> ...]   (default SUBSTR: mlp_train)"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(argv):
    sub = "mlp_train"
    if argv[:1] == ["--kernel"]:
        sub, argv = argv[1], argv[2:]
    per = defaultdict(lambda: defaultdict(list))
    for d in argv:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                per[name][(row["Counter_Name"], row.get("Dispatch_Id", ""))].append(float(row["Counter_Value"]))
    for name, cs in sorted(per.items()):
        if sub not in name:
            continue
        tot = defaultdict(list)
        for (c, _), v in cs.items():
            tot[c].append(sum(v))
        print(name)
        for c in sorted(tot):
            vals = tot[c]
            print(f"  {c:28s} {sum(vals) / len(vals):16.4g}  (n={len(vals)})")


if __name__ == "__main__":
    main(sys.argv[1:])
