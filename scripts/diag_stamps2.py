#!/usr/bin/env python3
"""Per-phase cycle breakdown of k_upd2 (cfg2: PPO Humanoid O=376, A=17, E=1024, T=2048, 32
minibatches -> M=65 536) from the diagnostic stamps build (make -C ppo.cpp_amd stamps). Runs one
cfg2 iteration (the stamps hold the last minibatch's launch) and prints, per trunk, the median
shader-clock cycles of each phase over waves and tiles, and the co-resident view: per CU, how
long each tile took with the other workgroup's waves beside it. Optional argument: save the raw
stamps ([wg, wave, tile, start + 12 phase ends + hardware id], uint64)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PPO_HIP_LIB"] = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import numpy as np  # noqa: E402

import ppo_amd  # noqa: E402

NAMES = ["top wait+bar", "L1 mm (384 K)", "tanh+H1 st+bar", "L2 mm+tanh+bar", "heads+bar", "loss1+crit+bar",
         "surrogate+bar", "rowdma+loss2+bar", "head bwd", "dz2+st+2bar", "dh1 mm", "dz1+st+cs"]
NP = len(NAMES)
NS, NT = NP + 2, 16
T = int(os.environ.get("CFG2_T", "2048"))
cfg = ppo_amd.PPOConfig(env_id="Humanoid-v4", num_envs=1024, num_steps=T, num_minibatches=32 * T // 2048,
                        update_epochs=1, total_timesteps=1024 * T * 4)
opts = os.environ.get("PPO_OPTS") or None
tr = ppo_amd.Trainer(cfg, options=opts)
tr.iterate()
tr.agent.sync()
lib = ppo_amd.lib()
n = 512 * 4 * NT * NS
buf = (C.c_ulonglong * n)()
lib.ppo_diag_read_stamps2.restype = C.c_int
lib.ppo_diag_read_stamps2(buf, C.c_long(n))
raw = np.frombuffer(buf, dtype=np.uint64).reshape(512, 4, NT, NS).copy()
if len(sys.argv) > 1:
    np.save(sys.argv[1], raw)
st = raw[..., :NP + 1].astype(np.int64)
ok = (st[..., 0] > 0)
d = np.diff(st, axis=-1)
for trunk, waves in (("critic", [0, 1]), ("actor", [2, 3])):
    x = d[:, waves][ok[:, waves]]
    x = x[(x >= 0).all(axis=1) & (x < 10**7).all(axis=1)]
    med = np.median(x, axis=0)
    tot = med.sum()
    print(f"{trunk}: {len(x)} wave-tiles, median tile {tot:.0f} cycles")
    for k, nm in enumerate(NAMES):
        print(f"  {k:2d} {nm:18s} {med[k]:8.0f}  {100 * med[k] / tot:5.1f}%")
# whole-workgroup tile time (start of tile to end of tile, wave 0) and the launch span
t0 = st[..., 0][ok]
t1 = st[..., NP][ok]
print(f"tile span median {np.median(t1 - t0):.0f} cycles; launch span {t1.max() - t0.min()} cycles over "
      f"{ok[:, 0].sum(axis=1).max()} tiles per workgroup")
# co-residency: workgroups sharing a CU (same SE/CU/XCC in the hardware id, bits of HW_ID)
hw = raw[..., NP + 1]
cu_key = ((hw[:, 0, 0] >> 8) & 0xFF) | (((hw[:, 0, 0] >> 32) & 0xF) << 8)  # HW_ID cu/sh/se bits + XCC id
print(f"distinct CU keys among workgroups: {len(set(cu_key.tolist()))} (of {raw.shape[0]} workgroups)")
tr.close()
