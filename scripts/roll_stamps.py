#!/usr/bin/env python3
"""Phase timing of the persistent rollout kernels (diagnostic stamps build, ROLL_STAMP in
csrc/ppo_rollout.hip): runs one rollout per config with libppo_hip_stamps.so and prints the mean
shader-clock cycles per phase over steps 1..15 of workgroup 0:
  k_rollout  (AC):  0 inputs | 1 trunk (L1, LN, L2, LN, heads; split into sub-phases) | 2 Beta sample /
                    actions | 3 env step
  k_rollout4 (PPO): 0 inputs + draws | 1 trunk (L1, L2) | 2 heads + actions + log-probs | 3 env + wrappers"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PPO_HIP_LIB"] = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import numpy as np  # noqa: E402
import ppo_amd  # noqa: E402


def run(name, cfg):
    tr = ppo_amd.Trainer(cfg)
    tr.rollout()
    tr.agent.sync()
    buf = (C.c_ulonglong * 128)()
    n = ppo_amd.lib().ppo_diag_read_roll_stamps(buf, 128)
    full = np.array(buf[:n], np.int64).reshape(16, 8)[1:]
    st = full[:, :5]
    d = np.diff(st, axis=1).mean(0)
    if name.startswith("ac"):  # k_rollout's trunk: L1 + LayerNorm 1 | layer-2 MFMAs | LayerNorm 2 | heads
        sub = np.stack([full[:, 5] - full[:, 1], full[:, 6] - full[:, 5], full[:, 7] - full[:, 6],
                        full[:, 2] - full[:, 7]], 1).mean(0)
        print(name, "trunk sub-phases [L1+LN1, L2 mm, LN2, heads]", np.round(sub, 1).tolist(), flush=True)
    # s_memtime counts shader clock cycles (22 K per AC step at E = 512 = 9.3 us at 2.4 GHz)
    print(name, "E", cfg.num_envs, "per-step cycles", st[:, 4].mean() - st[:, 0].mean(),
          "phases", np.round(d, 1).tolist(), flush=True)
    tr.close()


ppo_amd.set_device(0)
ppo_amd.lib().ppo_diag_read_roll_stamps.argtypes = [C.c_void_p, C.c_long]
run("ac_halfcheetah", ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=512, num_steps=16, total_timesteps=512 * 16 * 4))
run("ppo_humanoid", ppo_amd.PPOConfig(env_id="Humanoid-v4", num_envs=1024, num_steps=16, total_timesteps=1024 * 16 * 4))
run("ppo_halfcheetah_e1", ppo_amd.PPOConfig(env_id="HalfCheetah-v5", num_envs=1, num_steps=64, total_timesteps=64 * 4))
