"""Effective shader clock per kernel from a rocprofv3 GRBM_GUI_ACTIVE pass
(MI355X_MICROARCH.md 'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time;
reads high on dispatches shorter than ~0.3 ms).
usage: python tools/clock_summary.py <run_counter_collection.csv>"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
groups = {"train critic (k_mlp_train_x3<0, G13)": ("k_mlp_train_x3<0", "Geo<16, 1, 13"),
          "train actor (k_mlp_train_x3<1, G13)": ("k_mlp_train_x3<1", "Geo<16, 1, 13"),
          "env step (k_sample_env_r)": ("k_sample_env_r",), "policy (k_policy_mfma)": ("k_policy_mfma",)}
for name, pat in groups.items():
    v = []
    for r in rows:
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and all(p in r["Kernel_Name"] for p in pat):
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            v.append((float(r["Counter_Value"]) / 8 / dur / 1e9, dur * 1e3))
    if not v:
        continue
    c = [x[0] for x in v]
    print(f"{name}: {len(v)} dispatches, effective clock median {st.median(c):.3f} GHz (min {min(c):.3f}, "
          f"max {max(c):.3f}; last 20 median {st.median(c[-20:]):.3f}), wall median {st.median([x[1] for x in v]):.4f} ms")
