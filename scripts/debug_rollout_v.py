#!/usr/bin/env python3
"""Debug aid: where does the VALU persistent rollout (rollout_kernel=valu) first differ from the MFMA
one and from the per-step path? Prints, per stored buffer and step, the count and max |diff|."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RDBG = os.environ.get("RDBG") == "1"  # also the per-layer dumps of env 26 at step 0 (g_rdbg)
# the diagnostic build (make -C ppo.cpp_amd stamps): ppo_debug_buffer, ppo_diag_read_rdbg
os.environ["PPO_HIP_LIB"] = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import numpy as np  # noqa: E402

import ppo_amd  # noqa: E402

E, T = int(os.environ.get("DBG_E", "200")), 8
cfg = ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=E, num_steps=T, num_minibatches=4, update_epochs=1,
                          total_timesteps=E * T * 4)
BUFS = [("obs", "BUF_OBS", 1), ("actions", "BUF_ACTIONS", 2), ("logp", "BUF_LOGPROBS", 0), ("rewards", "BUF_REWARDS", 0),
        ("values", "BUF_VALUES", 0)]
res = {}
for name, opt in (("valu", "rollout_kernel=valu"), ("mfma", "rollout_kernel=mfma"), ("step", "rollout=per_step")):
    tr = ppo_amd.Trainer(cfg, options=opt)
    tr.rollout()
    tr.agent.sync()
    O, A = tr.hcfg.obs_dim, tr.hcfg.act_dim
    res[name] = {b: tr.agent.buffer(getattr(ppo_amd, k), (T, E, O) if kd == 1 else (T, E, A) if kd == 2 else (T, E)).numpy()
                 for b, k, kd in BUFS}
    import ctypes
    lib = ppo_amd.lib()
    lib.ppo_debug_buffer.restype = ctypes.c_void_p
    lib.ppo_debug_buffer.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    bp = lib.ppo_debug_buffer(tr.agent.h, b"beta_store")
    if bp:
        res[name]["beta"] = ppo_amd.DeviceArray.wrap(bp, (T, E, A, 3)).numpy()
    tr.close()
for a, b in (("mfma", "step"), ("valu", "step"), ("valu", "mfma")):
    for k in [k for k in res[a] if k in res[b]]:
        for t in range(T):
            d = np.abs(res[a][k][t].astype(np.float64) - res[b][k][t])
            n = int((res[a][k][t] != res[b][k][t]).sum())
            if n:
                idx = np.unravel_index(np.argmax(d), d.shape)
                print(f"{a} vs {b} {k} t={t}: {n} differ, max {d.max():.3e} at {idx}: {res[a][k][t][idx]!r} vs {res[b][k][t][idx]!r}")
                break
if "beta" in res["valu"] and "beta" in res["mfma"]:
    bv, bm = res["valu"]["beta"], res["mfma"]["beta"]
    for q, nm in enumerate(("alpha", "beta", "s01")):
        d = bv[..., q] != bm[..., q]
        print(nm, "differ:", int(d.sum()), "first at", [tuple(int(v) for v in x) for x in np.argwhere(d)[:4]])
    t0 = np.argwhere(bv[0, :, :, 0] != bm[0, :, :, 0])
    for e, a in t0[:6]:
        print("t=0 env", e, "action", a, "valu", bv[0, e, a].tolist(), "mfma", bm[0, e, a].tolist())
if RDBG:
    import ctypes
    lib = ppo_amd.lib()
    buf = (ctypes.c_float * 2560)()
    lib.ppo_diag_read_rdbg(buf)
    d = np.frombuffer(buf, dtype=np.float32).reshape(2, 1280)
    for nm, lo, n in (("l1", 0, 256), ("h1", 260, 256), ("l2", 516, 256), ("h2", 776, 256), ("hp", 1032, 128),
                      ("pre", 1160, 12)):
        m, v = d[0, lo:lo + n], d[1, lo:lo + n]
        bad = np.nonzero(m != v)[0]
        print(f"rdbg {nm}: {len(bad)} differ", [(int(i), float(m[i]), float(v[i])) for i in bad[:5]])
print("done")
