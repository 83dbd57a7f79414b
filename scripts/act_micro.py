#!/usr/bin/env python3
"""Micro-benchmark of one rollout act launch (ppo_rollout_act) and of the API forward
(ppo_get_action_and_value, no rollout stores) for the PPO (H = 64 tanh) and AC (H = 256 LN)
agents at several E, HIP-event timed over back-to-back launches on the context stream.
Prints one JSON line per case (us per launch)."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ppo.cpp_amd"))
import ppo_amd  # noqa: E402
from ppo_amd import DeviceArray, lib  # noqa: E402

hip = C.CDLL("libamdhip64.so")


def time_launches(fn, stream, n=200):
    ev0, ev1 = C.c_void_p(), C.c_void_p()
    hip.hipEventCreate(C.byref(ev0)); hip.hipEventCreate(C.byref(ev1))
    for _ in range(20):
        fn()
    hip.hipEventRecord(ev0, C.c_void_p(stream))
    for _ in range(n):
        fn()
    hip.hipEventRecord(ev1, C.c_void_p(stream))
    hip.hipEventSynchronize(ev1)
    ms = C.c_float()
    hip.hipEventElapsedTime(C.byref(ms), ev0, ev1)
    return ms.value * 1e3 / n


def main():
    ppo_amd.set_device(0)
    lib().ppo_stream.restype = C.c_void_p
    cases = [(0, 376, 17, 64), (0, 17, 6, 64), (1, 17, 6, 256), (1, 105, 8, 256)]
    if os.environ.get("ACT_MICRO_CASES"):  # e.g. "1,17,6,256;0,376,17,64"
        cases = [tuple(int(v) for v in c.split(",")) for c in os.environ["ACT_MICRO_CASES"].split(";")]
    for kind, O_, A, H in cases:
        for E in (64, 512, 1024, 4096):
            hc = ppo_amd.HipConfig(kind, O_, A, H, E, 4, 1, 1, 0.99, 0.95, 0.2, 0.01, 0.5, 0.5, 1e-5, 1, 1, 1, 0, 1)
            ag = ppo_amd.Agent(hc)
            rng = np.random.default_rng(0)
            x = DeviceArray.from_numpy(rng.standard_normal((E, O_)).astype(np.float32))
            d = DeviceArray.from_numpy(np.zeros(E, np.float32))
            act = DeviceArray((E, A)); lp = DeviceArray(E); ent = DeviceArray(E); val = DeviceArray(E)
            s = lib().ppo_stream(ag.h)
            t_roll = time_launches(lambda: lib().ppo_rollout_act(ag.h, 0, 0, E, x.ptr, d.ptr, act.ptr, None), s)
            t_api = time_launches(lambda: lib().ppo_get_action_and_value(ag.h, E, x.ptr, 0, None, 0, 0, act.ptr, lp.ptr,
                                                                        ent.ptr, val.ptr, None), s)
            t_val = time_launches(lambda: lib().ppo_get_value(ag.h, E, x.ptr, val.ptr, None), s)
            print(json.dumps({"diag": os.environ.get("PPO_ACT_DIAG", ""), "kind": kind, "O": O_, "A": A, "H": H, "E": E, "rollout_act_us": round(t_roll, 2),
                              "api_act_us": round(t_api, 2), "get_value_us": round(t_val, 2)}), flush=True)
            ag.close()


if __name__ == "__main__":
    main()
