#!/usr/bin/env python3
"""Per-launch durations of the last CaRL update in a rocprofv3 kernel trace (scripts/bench_carla.py)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
idx = [i for i, r in enumerate(rows) if "k_carla_adam" in r["Kernel_Name"]]
a, b = (idx[-2] + 1, idx[-1] + 1) if len(idx) > 1 else (0, len(rows))
tot = 0.0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    wg = int(r["Workgroup_Size_X"]) or 1
    print(f"{name:24s} grid=({int(r['Grid_Size_X']) // wg},{r['Grid_Size_Y']},{r['Grid_Size_Z']}) {d:9.1f} us")
print(f"total {tot / 1e3:.2f} ms")
