"""Idle time between consecutive kernels in a rocprofv3 kernel trace (one GPU, one stream).

    python3 scripts/kernel_gaps.py <dir with *kernel_trace.csv> [--name-width 24]

Prints, per transition (previous kernel -> next kernel), the count and the median / mean / max
gap in microseconds, and per iteration (delimited by k_gae launches) the busy time (sum of kernel
durations) against the span from the first start to the last end. Used to decide whether the
rollout's 2 x 128 launches per iteration lose time between kernels.
"""
import csv
import glob
import os
import statistics
import sys


def short(name, w):
    n = name.split("(")[0].replace("void ", "")
    return n[:w]


def main():
    d = sys.argv[1]
    w = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--name-width" else 24
    files = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"], w)))
    rows.sort()
    trans = {}
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        trans.setdefault((n0, n1), []).append((s1 - e0) / 1e3)
    print(f"{'previous':<{w}} {'next':<{w}} {'count':>6} {'med_us':>8} {'mean_us':>8} {'max_us':>8}")
    for (a, b), g in sorted(trans.items(), key=lambda kv: -len(kv[1])):
        print(f"{a:<{w}} {b:<{w}} {len(g):>6} {statistics.median(g):>8.2f} {statistics.mean(g):>8.2f} {max(g):>8.2f}")
    # iterations: from one k_gae to the next (rollout of the next iteration precedes its k_gae)
    gae = [i for i, r in enumerate(rows) if r[2].startswith("k_gae")]
    print("\niteration (k_gae to k_gae): busy_ms span_ms idle_frac")
    for a, b in zip(gae, gae[1:]):
        seg = rows[a:b]
        busy = sum(e - s for s, e, _ in seg) / 1e6
        span = (rows[b][0] - rows[a][0]) / 1e6
        print(f"  {busy:8.3f} {span:8.3f} {1 - busy / span:6.3f}")


if __name__ == "__main__":
    main()
