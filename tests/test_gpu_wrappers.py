"""The PPO env wrapper chain on the device (ppo_continuous_action.cpp:41-49,
stateful_observation.h:56-84, stateful_reward.h:55-91) through include/ppo_env_wrappers.h.

  * pwrap_step (its own kernel) fed the raw stream of the golden case's scripted env (termination,
    truncation, next-step autoreset, a plain reset mid-episode, both clamps) in several envs at
    once: bit-exact against the oracle's vector chain, observations within 1 ulp of the LibTorch
    replay (its CPU torch::sqrt is not correctly rounded, see test_wrappers.py), rewards and the
    final statistics bit-exact against the golden vectors.
  * the chain fused into the synthetic device env's kernels (psyn_attach_wrappers; the narrow
    k_synth_step and the wide k_synth_step_wide) over 1 005 steps, through the 1 000-step
    truncation and its autoreset: bit-exact against the oracle env with the oracle chain on top.
"""
import numpy as np
import pytest

import oracle_lib as O
from golden_io import load_case

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402


def test_device_chain_vs_golden_and_oracle():
    meta, d = load_case("wrappers")
    Od, T, gamma = meta["O"], meta["T"], meta["gamma"]
    raw, r, te, tr, rs = O.wrappers_script(Od, T, meta["reset_at"])
    E = 5
    w = ppo_amd.EnvWrappers(E, Od, gamma)
    ow = O.VecWrappers(E, Od, gamma)
    obs = DeviceArray.from_numpy(np.tile(raw[0], (E, 1)))
    w.reset(obs)
    np.testing.assert_array_equal(obs.numpy(), ow.reset(np.tile(raw[0], (E, 1))))
    np.testing.assert_array_max_ulp(obs.numpy()[0], d["obs"][0], maxulp=1)
    for t in range(T):
        o_in = np.tile(raw[t + 1], (E, 1))
        r_in, te_in, rs_in = (np.full(E, x[t], np.float32) for x in (r, te, rs))
        obs = DeviceArray.from_numpy(o_in)
        rew = DeviceArray.from_numpy(r_in)
        w.step(obs, rew, DeviceArray.from_numpy(te_in), DeviceArray.from_numpy(rs_in))
        oo, orw = ow.step(o_in, r_in, te_in, rs_in)
        np.testing.assert_array_equal(obs.numpy(), oo, err_msg=f"step {t}")
        np.testing.assert_array_equal(rew.numpy(), orw, err_msg=f"step {t}")
        np.testing.assert_array_max_ulp(obs.numpy()[E - 1], d["obs"][t + 1], maxulp=1)
        np.testing.assert_array_equal(rew.numpy()[E - 1], d["reward"][t])
    st, ost = w.state(), ow.state()
    for k in st:
        np.testing.assert_array_equal(st[k], ost[k], err_msg=k)
    np.testing.assert_array_equal(st["obs_mean"][0], d["obs_mean_final"])
    np.testing.assert_array_equal(st["obs_var"][3], d["obs_var_final"])
    w.close()


@pytest.mark.parametrize("O_,A", [(17, 6), (105, 8), (376, 17)])
def test_fused_chain_in_device_env_vs_oracle(O_, A):
    E = 300
    env = ppo_amd.SynthEnv(E, O_, A)
    w = ppo_amd.EnvWrappers(E, O_, 0.99)
    env.attach_wrappers(w)
    oenv = O.SynthEnv(E, O_, A, wrappers=True, gamma=0.99)
    obs = DeviceArray((E, O_)); done = DeviceArray(E); rew = DeviceArray(E)
    env.reset(7, obs, done)
    np.testing.assert_array_equal(obs.numpy(), oenv.reset(7))
    rng = np.random.default_rng(1)
    for t in range(1005):
        a = rng.uniform(-1.3, 1.3, (E, A)).astype(np.float32)
        env.step(DeviceArray.from_numpy(a), obs, rew, done)
        o_obs, o_r, o_te, o_tr, _, _ = oenv.step(a)
        if t % 97 == 0 or t >= 998:
            np.testing.assert_array_equal(obs.numpy(), o_obs, err_msg=f"step {t}")
            np.testing.assert_array_equal(rew.numpy(), o_r, err_msg=f"step {t}")
            np.testing.assert_array_equal(done.numpy(), np.maximum(o_te, o_tr))
    st, ost = w.state(), oenv.wrap.state()
    for k in st:
        np.testing.assert_array_equal(st[k], ost[k], err_msg=k)
    assert np.abs(obs.numpy()).max() <= 10.0
    sr, sl, n = env.episode_stats()  # RecordEpisodeStatistics sits inside the chain: raw returns
    assert n == E
    env.close()
    w.close()
