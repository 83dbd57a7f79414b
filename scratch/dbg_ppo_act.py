import sys, os
sys.path.insert(0, "ppo.cpp_amd"); sys.path.insert(0, "tests")
import numpy as np, ppo_amd
from ppo_amd import DeviceArray
from golden_io import load_case
import oracle_lib as O
meta, d = load_case("ppo_act")
n = 64
hc = ppo_amd.HipConfig(0, 17, 6, 64, n, 1, 1, 1, 0.99, 0.95, 0.2, 0.0, 0.5, 0.5, 1e-5, 1, 1, 1, 0, 1)
ag = ppo_amd.Agent(hc)
ag.load_params(d["params"])
x = DeviceArray.from_numpy(d["x"]); a = DeviceArray.from_numpy(d["action"])
for mode in (2, 1, 0):
    act, lp, ent, v = ag.get_action_and_value(x, mode, a if mode == 2 else None)
    print("mode", mode, "lp", lp.numpy()[:4], "ent", ent.numpy()[:4], "v", v.numpy()[:4], "act", act.numpy()[0])
print("golden lp", d["logprob"][:4], "ent", d["entropy"][:4], "v", d["value"][:4], "mean", d["mean"][0])
