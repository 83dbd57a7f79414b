#!/usr/bin/env python3
"""Timeline of one rollout act launch (k_act3) from the diagnostic stamps build
(make -C ppo.cpp_amd stamps): per trunk, median shader-clock time of each phase end relative to
the earliest wave start of the launch, and the spread of wave start times (dispatch skew)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PPO_HIP_LIB"] = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import numpy as np  # noqa: E402

import ppo_amd  # noqa: E402

NAMES = ["start", "inputs+bar", "L1 mm", "LN1", "st+bar", "L2 mm", "LN2", "heads+bar", "PRE+bar",
         "dist stage1+bar", "dist stage2+bar", "end"]
NS = 12
cfg = ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=4096, num_steps=128, total_timesteps=4096 * 128 * 4)
tr = ppo_amd.Trainer(cfg, num_envs_per_device=4096)
tr.iterate()
# the stamps keep the last launch: end on a rollout act (actor + critic), not the critic-only
# GAE bootstrap
tr.rollout()
tr.agent.sync()
lib = ppo_amd.lib()
n = 512 * 8 * NS
buf = (C.c_ulonglong * n)()
got = lib.ppo_diag_read_act_stamps(buf, C.c_long(n))
st = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(512, 8, NS)
t0 = st[:, :, 0][st[:, :, 0] > 0].min()
for trunk, sl in (("critic", slice(0, 128)), ("actor", slice(256, 384))):
    x = st[sl].reshape(-1, NS)
    x = x[x[:, 0] > 0]
    rel = x - t0
    print(f"{trunk}: {len(x)} waves; start spread p10/p50/p90 = {np.percentile(rel[:, 0], [10, 50, 90]).astype(int)}")
    for k, nm in enumerate(NAMES):
        col = rel[:, k]
        col = col[(col >= 0) & (col < 10**7)]
        if len(col):
            print(f"  {k:2d} {nm:16s} p50 {np.median(col):8.0f}  p90 {np.percentile(col, 90):8.0f}")
tr.close()
