#!/usr/bin/env python3
"""Pair each critic wave of k_upd with the actor wave on the same SIMD (hardware ids recorded by the
stamps build, scripts/diag_stamps.py OUT.npy) and report, per phase of each trunk, how the
partner's time splits over its phases: which phases actually run side by side on a SIMD."""
import sys

import numpy as np

NAMES = ["top", "L1mm", "LN1", "L2mm", "LN2", "heads", "PRE", "loss", "hbwd", "LN2bwd", "dh1mm", "L1re", "LN1bwd"]
NP = len(NAMES)
raw = np.load(sys.argv[1]).astype(np.int64)  # [1024 wg, 4 wave, 16 tile, 15]
hw = raw[..., NP + 1]
key = ((hw & 0xFFFFFFFF) >> 4) & 0xFFF | ((hw >> 32) << 12)  # simd, pipe, cu, sh, se | xcc
key = np.where(raw[..., 0] > 0, key, -1)


def intervals(wg, w):
    out = []
    for t in range(16):
        st = raw[wg, w, t, :NP + 1]
        if st[0] <= 0 or (st[1:] <= 0).any():
            continue
        for p in range(NP):
            out.append((st[p], st[p + 1], p))
    return out


ov = np.zeros((2, NP, NP + 1))  # [trunk, own phase, partner phase or idle]
npair = 0
crit = {}
for wg in range(256):
    for w in range(4):
        k = key[wg, w, 2]
        if k >= 0:
            crit.setdefault(int(k), (wg, w))
for wg in range(512, 768):
    for w in range(4):
        k = int(key[wg, w, 2])
        if k < 0 or k not in crit:
            continue
        cw = crit[k]
        A, C = intervals(wg, w), intervals(*cw)
        if not A or not C:
            continue
        npair += 1
        for own, oth, tr in ((C, A, 0), (A, C, 1)):
            ob = np.array([x[0] for x in oth]); oe = np.array([x[1] for x in oth]); op = np.array([x[2] for x in oth])
            for s, e, p in own:
                cov = np.clip(np.minimum(oe, e) - np.maximum(ob, s), 0, None)
                np.add.at(ov[tr, p], op, cov)
                ov[tr, p, NP] += (e - s) - cov.sum()
print(f"{npair} SIMD pairs")
for tr, nm in ((0, "critic"), (1, "actor")):
    tot = ov[tr].sum(axis=1)
    print(f"{nm}: phase total (Mcycles summed over pairs) and partner's phase mix (%)")
    print(" " * 16 + " ".join(f"{n[:6]:>6s}" for n in NAMES) + "   idle")
    for p in range(NP):
        mix = 100 * ov[tr, p] / max(tot[p], 1)
        print(f"  {NAMES[p]:7s} {tot[p] / npair / 16:6.0f} " + " ".join(f"{m:6.1f}" for m in mix))
