"""Effective shader clock of every 13-input train launch, in order, per iteration (iterations split
at the k_choice dispatch), from a rocprofv3 GRBM_GUI_ACTIVE pass (clock = GRBM_GUI_ACTIVE / 8 XCDs /
dispatch wall, as tools/clock_summary.py).  usage: python tools/clock_sequence.py <run_counter_collection.csv>"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
it, seq = 0, []
for r in rows:
    n = r["Kernel_Name"]
    if "k_choice" in n:
        if seq:
            print(f"iter {it}: " + " ".join(seq))
        it, seq = it + 1, []
    elif "k_mlp_train_x3<" in n and "Geo<16, 1, 13" in n:
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        ghz = float(r["Counter_Value"]) / 8 / dur / 1e9
        seq.append(f"{'A' if 'x3<1' in n else 'C'}{dur * 1e3:.3f}ms@{ghz:.2f}")
if seq:
    print(f"iter {it}: " + " ".join(seq))
