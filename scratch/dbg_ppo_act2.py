import sys
sys.path.insert(0, "ppo.cpp_amd"); sys.path.insert(0, "tests")
import numpy as np, ppo_amd
from ppo_amd import DeviceArray
from golden_io import load_case
meta, d = load_case("ppo_act")
n = 64
hc = ppo_amd.HipConfig(0, 17, 6, 64, n, 1, 1, 1, 0.99, 0.95, 0.2, 0.0, 0.5, 0.5, 1e-5, 1, 1, 1, 0, 1)
ag = ppo_amd.Agent(hc)
ag.load_params(d["params"])
x = DeviceArray.from_numpy(d["x"])
for name, act_in in (("golden_action", d["action"]), ("mean", d["mean"]), ("mean+1", d["mean"] + 1), ("zeros", np.zeros((64, 6), np.float32))):
    a = DeviceArray.from_numpy(np.ascontiguousarray(act_in, np.float32))
    act, lp, ent, v = ag.get_action_and_value(x, 2, a)
    print(name, "lp", lp.numpy()[:3], "act_out", act.numpy()[0, :3], "act_in", act_in[0, :3])
# AC net same thing
meta, d = load_case("ac_act")
hc = ppo_amd.HipConfig(1, 17, 6, 64, n, 1, 1, 1, 0.99, 0.95, 0.2, 0.0, 0.5, 0.5, 1e-5, 1, 1, 1, 0, 1)
ag = ppo_amd.Agent(hc); ag.load_params(d["params"])
x = DeviceArray.from_numpy(d["x"]); a = DeviceArray.from_numpy(d["action"])
act, lp, ent, v = ag.get_action_and_value(x, 2, a)
print("AC lp", lp.numpy()[:3], d["logprob"][:3], "ent", ent.numpy()[:3], d["entropy"][:3], "v", v.numpy()[:3], d["value"][:3])
