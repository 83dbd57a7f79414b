#!/usr/bin/env python3
"""Per-launch durations of the last CaRL update in a rocprofv3 kernel trace (scripts/bench_carla.py);
with a second argument "forward", of the last forward (from the last conv1 launch to the end)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
if len(sys.argv) > 2 and sys.argv[2] == "forward":
    idx = [i for i, r in enumerate(rows) if "k_conv_img" in r["Kernel_Name"]]
    a, b = idx[-1], len(rows)
else:
    idx = [i for i, r in enumerate(rows) if "k_carla_adam" in r["Kernel_Name"]]
    a, b = (idx[-2] + 1, idx[-1] + 1) if len(idx) > 1 else (0, len(rows))
t_first = int(rows[a]["Start_Timestamp"])
tot = 0.0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    wg = int(r["Workgroup_Size_X"]) or 1
    print(f"{name:24s} grid=({int(r['Grid_Size_X']) // wg},{r['Grid_Size_Y']},{r['Grid_Size_Z']}) {d:9.1f} us")
print(f"total {tot / 1e3:.3f} ms busy, {(int(rows[b - 1]['End_Timestamp']) - t_first) / 1e6:.3f} ms first start -> last end")
