#!/usr/bin/env python3
"""Mean counter value per launch, per kernel class, over every *counter_collection.csv in a dir."""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import klass  # noqa: E402


def main():
    acc = {}
    for fn in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                k = klass(row.get("Kernel_Name", ""))
                if k is None:
                    continue
                key = (k, row["Counter_Name"])
                d = acc.setdefault(key, {})
                disp = row.get("Dispatch_Id") or row.get("Correlation_Id")
                d[disp] = d.get(disp, 0.0) + float(row["Counter_Value"])
    for (k, c) in sorted(acc):
        v = acc[(k, c)]
        print(f"{k:10s} {c:32s} {sum(v.values()) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
