#!/usr/bin/env python3
"""Overlap of GPU inference with CPU env stepping in the AC CLI's async host-env collection (cfg3),
from a rocprofv3 --kernel-trace --marker-trace run (scripts/async_sps.sh): every act kernel
(k_act*) and every blit of the per-step transfers (__amd_rocclr_copyBuffer) against the
"host_env_step" roctx ranges the collection threads open around their env stepping.

Reports, over the collection phases (first to last act kernel of each iteration):
  - the fraction of act-kernel time during which at least one OTHER thread is stepping envs
    (1.0 = the GPU inference is entirely hidden under CPU stepping),
  - per-thread CPU stepping time vs the phase's wall time (how busy the collection threads keep
    the host), and the GPU's busy fraction in the phase.
    python3 scripts/async_overlap.py <trace dir>
"""
import bisect
import csv
import glob
import os
import sys


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(d):
    kt = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0])))
    mk = list(csv.DictReader(open(glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True)[0])))
    steps = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Thread_Id"])) for r in mk
             if r["Function"] == "host_env_step"]
    acts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Thread_Id"])) for r in kt
            if r["Kernel_Name"].startswith("void k_act")]
    blits = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Thread_Id"])) for r in kt
             if "copyBuffer" in r["Kernel_Name"]]
    upds = sorted(int(r["Start_Timestamp"]) for r in kt if r["Kernel_Name"].startswith("void k_upd"))
    # collection phases: act kernels between consecutive update blocks
    acts.sort()
    phases, cur = [], []
    ui = 0
    for a in acts:
        while ui < len(upds) and upds[ui] < a[0]:
            ui += 1
            if cur:
                phases.append(cur)
                cur = []
        cur.append(a)
    if cur:
        phases.append(cur)
    steps.sort()
    starts = [s for s, _, _ in steps]
    print(f"act kernels {len(acts)}, transfer blits {len(blits)}, host_env_step ranges {len(steps)}, "
          f"threads {len(set(t for _, _, t in steps))}")
    for pi, ph in enumerate(phases):
        p0, p1 = ph[0][0], max(e for _, e, _ in ph)
        if len(ph) < 100:
            print(f"phase {pi}: {len(ph)} act kernels (evaluation / bootstrap), skipped")
            continue
        act_t = hidden_t = 0
        for s, e, th in ph:
            act_t += e - s
            # the union of other threads' stepping ranges within [s, e]
            j = bisect.bisect_left(starts, s - 50_000_000)
            cov = []
            for k in range(j, len(steps)):
                ss, se, st = steps[k]
                if ss > e:
                    break
                if st != th and se > s:
                    cov.append((max(ss, s), min(se, e)))
            hidden_t += union_len(cov)
        ph_steps = [(s, e, t) for s, e, t in steps if s >= p0 - 1_000_000 and e <= p1 + 5_000_000]
        if not ph_steps:
            print(f"phase {pi}: {len(ph)} act kernels without host stepping ranges (evaluation), skipped")
            continue
        threads = sorted(set(t for _, _, t in ph_steps))
        wall = max(e for _, e, _ in ph_steps) - min(s for s, _, _ in ph_steps)
        per_thread = [sum(e - s for s, e, t in ph_steps if t == th) for th in threads]
        gpu = [(s, e) for s, e, _ in ph] + [(s, e) for s, e, _ in blits if p0 <= s <= p1]
        print(f"phase {pi}: wall {wall / 1e6:.2f} ms, {len(ph)} act kernels = {act_t / 1e6:.2f} ms of kernel time, "
              f"{hidden_t / act_t:.3f} of it under another thread's env stepping; host stepping per thread "
              f"{min(per_thread) / 1e6:.1f}-{max(per_thread) / 1e6:.1f} ms of the {wall / 1e6:.1f} ms "
              f"(mean {sum(per_thread) / len(per_thread) / wall:.3f} busy, {len(threads)} threads); GPU busy "
              f"{union_len(gpu) / (p1 - p0):.3f} of the phase (act + transfer blits)")


if __name__ == "__main__":
    main(sys.argv[1])
