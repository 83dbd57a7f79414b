#!/usr/bin/env python3
"""Micro-benchmark of the act kernel at E=4096 (AC HalfCheetah agent): per-mode launch time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import ppo_amd  # noqa: E402
from ppo_amd import DeviceArray  # noqa: E402
import oracle_lib as O  # noqa: E402

E, N = int(os.environ.get("E", "4096")), 300
L = O.layout_init(1, 17, 6, 256)
rng = np.random.default_rng(0)
p = (rng.standard_normal(L.P) * 0.05).astype(np.float32)
p[L.hi], p[L.lo] = 1.0, -1.0
p[L.ostd:L.ostd + 17] = 1.0
hc = ppo_amd.HipConfig(1, 17, 6, 256, E, 8, 1, 1, 0.99, 0.95, 0.1, 0.01, 0.5, 0.5, 1e-5, 1, 1, 1, 0, 1)
ag = ppo_amd.Agent(hc)
ag.load_params(p)
x = DeviceArray.from_numpy(rng.standard_normal((E, 17)).astype(np.float32))
a_in = DeviceArray.from_numpy(rng.uniform(-0.9, 0.9, (E, 6)).astype(np.float32))
res = {}
lib = ppo_amd.lib()
act = DeviceArray((E, 6)); lp = DeviceArray(E); ent = DeviceArray(E); val = DeviceArray(E)


def gav(mode, ain=None, step=0):
    lib.ppo_get_action_and_value(ag.h, E, x.ptr, mode, ain.ptr if ain else None, 0, step, act.ptr, lp.ptr, ent.ptr,
                                 val.ptr, None)


for name, fn in [("sample", lambda i: gav(ppo_amd.PPO_SAMPLE, step=i)),
                 ("mean", lambda i: gav(ppo_amd.PPO_MEAN)),
                 ("given", lambda i: gav(ppo_amd.PPO_GIVEN, a_in)),
                 ("value", lambda i: lib.ppo_get_value(ag.h, E, x.ptr, val.ptr, None))]:
    for i in range(10):
        fn(i)
    ag.sync()
    t0 = time.perf_counter()
    for i in range(N):
        fn(i)
    ag.sync()
    res[name] = round((time.perf_counter() - t0) / N * 1e6, 2)
print("E=%d us/launch" % E, res)
