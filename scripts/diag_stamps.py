#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_upd from the diagnostic stamps build (make -C ppo.cpp_amd stamps).
Runs one metric-config iteration (AC HalfCheetah, E=4096) and prints, per trunk, the median
shader-clock cycles of each phase over waves and tiles 2..13 of every workgroup. With an output
path argument it also saves the raw stamps ([wg, wave, tile, start + 13 phase ends + hardware id],
uint64) for scripts/corun_analysis.py."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PPO_HIP_LIB"] = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import numpy as np  # noqa: E402

import ppo_amd  # noqa: E402

NAMES = ["top+gather", "L1 mm", "LN1+st+bar", "L2 mm issue", "LN2", "heads+bar", "PRE+bar", "loss+bar",
         "hbias+head bwd", "LN2bwd+cs+st", "dh1 mm issue", "L1 re mm", "LN1bwd+cs+st"]
NP = len(NAMES)
NS, NT = NP + 2, 16
# --ant: the cfg4 shard (Ant-v5, E = 1 024, 32 768-row minibatches: 4 tiles per workgroup)
ANT = "--ant" in sys.argv
sys.argv = [x for x in sys.argv if x != "--ant"]
if ANT:
    cfg = ppo_amd.ACPPOConfig(env_id="Ant-v5", num_envs=1024, num_steps=128, total_timesteps=1024 * 128 * 4)
else:
    cfg = ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=4096, num_steps=128, total_timesteps=4096 * 128 * 4)
# PPO_OPTS: ppo_create_ex options (e.g. upd_mfma=32: the same phases of k_upd32)
tr = ppo_amd.Trainer(cfg, num_envs_per_device=cfg.num_envs, options=os.environ.get("PPO_OPTS") or None)
tr.iterate()
tr.agent.sync()
lib = ppo_amd.lib()
n = 1024 * 4 * NT * NS
buf = (C.c_ulonglong * n)()
lib.ppo_diag_read_stamps.restype = C.c_int
got = lib.ppo_diag_read_stamps(buf, C.c_long(n))
raw = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 4, NT, NS).copy()
if len(sys.argv) > 1:
    np.save(sys.argv[1], raw)
st = raw[..., :NP + 1].astype(np.int64)
d = np.diff(st, axis=-1)[:, :, (0 if ANT else 2):(4 if ANT else NT - 2)]  # [wg, wave, tile, phase]
for trunk, sl in (("critic", slice(0, 256)), ("actor", slice(512, 768))):
    x = d[sl].reshape(-1, NP)
    x = x[(x > 0).all(axis=1) & (x < 10**7).all(axis=1)]
    if not len(x):
        print(f"{trunk}: no tiles")
        continue
    med = np.median(x, axis=0)
    tot = med.sum()
    print(f"{trunk}: {len(x)} wave-tiles, median tile {tot:.0f} cycles")
    for k, nm in enumerate(NAMES):
        print(f"  {k:2d} {nm:16s} {med[k]:8.0f}  {100 * med[k] / tot:5.1f}%")
# co-residency: each workgroup's span (wave 0, first tile start .. last stamped tile end) and its CU
# (HW_ID bits 8..15: CU / SH / SE, XCC id in the upper word); the critic and actor workgroups of a CU
# run side by side only if their spans overlap
ntile = int(min(NT, (cfg.num_envs * cfg.num_steps // 4 + 31) // 32 // 256))
span0 = raw[:, 0, 0, 0].astype(np.int64)
span1 = raw[:, 0, ntile - 1, NP].astype(np.int64)
cuk = ((raw[:, 0, 0, NP + 1] >> np.uint64(8)) & np.uint64(0xFF)) | ((raw[:, 0, 0, NP + 1] >> np.uint64(32)) << np.uint64(8))
ok = (span0 > 0) & (span1 > span0)
wgs = [w for w in list(range(256)) + list(range(512, 768)) if ok[w]]
if wgs:
    t0 = min(span0[w] for w in wgs)
    print(f"launch span {max(span1[w] for w in wgs) - t0} cycles over {ntile} tiles per workgroup; "
          f"median workgroup span critic {np.median([span1[w] - span0[w] for w in wgs if w < 512]):.0f}, "
          f"actor {np.median([span1[w] - span0[w] for w in wgs if w >= 512]):.0f}")
    bycu = {}
    for w in wgs:
        bycu.setdefault(int(cuk[w]), []).append(w)
    ov = []
    for ws in bycu.values():
        c = [w for w in ws if w < 512]
        a_ = [w for w in ws if w >= 512]
        for wc in c:
            for wa in a_:
                inter = min(span1[wc], span1[wa]) - max(span0[wc], span0[wa])
                ov.append(max(0, inter) / max(span1[wc] - span0[wc], span1[wa] - span0[wa]))
    print(f"CU keys {len(bycu)}; critic/actor pairs on one CU {len(ov)}, "
          f"mean overlap of their spans {np.mean(ov) if ov else 0:.2f}; start offsets (median) "
          f"critic {np.median([span0[w] - t0 for w in wgs if w < 512]):.0f} actor {np.median([span0[w] - t0 for w in wgs if w >= 512]):.0f}")
tr.close()
