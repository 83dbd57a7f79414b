#!/usr/bin/env python3
"""Per-kernel HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts 64 B per memory-side read
request while wide coalesced reads issue 128-B requests, so it reports half the bytes: it is
doubled here. WRITE_SIZE is exact for 16-B-per-lane stores. Both counters are in KB (1024 B).
Usage: pmc_traffic.py <rocprof out dir> <config tag> [source label]  -> JSON on stdout."""
import csv
import glob
import json
import os
import re
import sys

CLASSES = [("k_fwdbwd", "fwdbwd"), ("k_upd", "fwdbwd"), ("k_dw", "dw"), ("k_act", "act"), ("k_colsum", "colsum"),
           ("k_gradnorm", "gradnorm"), ("k_adam", "adam"), ("k_gae", "gae"), ("k_perm", "perm"),
           ("k_adv_", "adv_stats"), ("k_synth_step", "synth_env"), ("k_rollout", "rollout"),
           ("k_values", "values"),
           # CaRL (cfg5) kernels
           ("k_conv_t", "conv2_fwd"), ("k_wgrad_t", "conv2_wgrad"), ("k_dgrad_q", "conv2_dgradq"),
           ("k_conv_img3", "conv1_fwd"), ("k_conv_img2", "conv1_fwd"), ("k_wgrad_img2", "conv1_wgrad"), ("k_dgrad_s2", "conv2_dgrad"),
           ("k_conv_fin", "conv_fin"), ("k_conv", "conv"), ("k_wgrad", "wgrad"), ("k_dgrad", "dgrad"),
           ("k_wsum", "wsum")]


def klass(name):
    for pat, k in CLASSES:
        if re.search(r"\b" + pat, name):
            return k
    return None


def per_kernel(path, counter):
    acc = {}
    for fn in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                k = klass(row.get("Kernel_Name", ""))
                if k is None:
                    continue
                key = (row.get("Dispatch_Id") or row.get("Correlation_Id"), k)
                acc.setdefault(k, {}).setdefault(key, 0.0)
                acc[k][key] += float(row["Counter_Value"])
    return {k: (sum(v.values()), len(v)) for k, v in acc.items()}


def main():
    path, tag = sys.argv[1], sys.argv[2]
    source = sys.argv[3] if len(sys.argv) > 3 else os.path.basename(os.path.normpath(path))
    fetch = per_kernel(os.path.join(path), "FETCH_SIZE")
    write = per_kernel(os.path.join(path), "WRITE_SIZE")
    out = {"_note": "bytes per launch; FETCH_SIZE doubled (gfx950 correction), KB = 1024 B; config = bench workload",
           "_source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of `bench.py --steps 1 --warmup 1`: {source}"}
    for k in sorted(set(fetch) | set(write)):
        fsum, fn = fetch.get(k, (0.0, 0))
        wsum, wn = write.get(k, (0.0, 0))
        if fn == 0 or wn == 0:
            continue
        rd = 2.0 * fsum * 1024 / fn
        wr = wsum * 1024 / wn
        out[k] = {"config": tag, "read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
                  "hbm_bytes_per_launch": round(rd + wr), "launches_fetch": fn, "launches_write": wn}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
