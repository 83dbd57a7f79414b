"""PPO env wrapper chain (ppo_continuous_action.cpp:41-49): the product's
gymcpp::make_env inside gymcpp::SeqVectorEnv and the oracle's restated Welford
(oracle/ppo_oracle.c orc_wrappers_run) against the LibTorch replay of stateful_observation.h:56-84 /
stateful_reward.h:55-91 (golden case `wrappers`, oracle/ref_harness.cpp), bit for bit.

The scripted env terminates every 29th call and truncates every 61st, so the run covers
termination, truncation, the next-step autoreset (reset(-1), reward 0; the observation statistics
update on it), a plain reset mid-episode, the discounted-return accumulator carried across resets
and both +-10 clamps (the reward clamp is hit while the reward variance is still tiny).

Tolerance: everything is bit-exact except the normalised observation, which may differ by 1 ulp.
LibTorch's CPU torch::sqrt (NormalizeObservation's sqrt(var_ + eps), stateful_observation.h:62)
is MKL VML's vsSqrt, which is not correctly rounded: on this Xeon it returns 1 ulp below the IEEE
result for ~0.65 % of inputs (measured with torch 2.10: 648 of 100 000). The Welford statistics
themselves contain no sqrt and stay bit-exact; the reward path uses std::sqrt on a float
(stateful_reward.h:75) and is bit-exact too."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from golden_io import load_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _oracle_run(Od, T, reset_at, gamma):
    obs = np.zeros((T + 1, Od), np.float32)
    out = {k: np.zeros(T, np.float32) for k in ("reward", "term", "trunc", "info_ret", "info_len")}
    mean, var = np.zeros(Od, np.float32), np.zeros(Od, np.float32)
    O.lib().orc_wrappers_run(Od, T, reset_at, C.c_float(gamma), O.fp(obs), *[O.fp(out[k]) for k in
                             ("reward", "term", "trunc", "info_ret", "info_len")], O.fp(mean), O.fp(var))
    return obs, out, mean, var


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("wrappers") / "wrappers_driver")
    subprocess.run(["g++", "-O2", "-std=c++20", "-ffp-contract=off", "-pthread",
                    os.path.join(ROOT, "tests", "native", "wrappers_driver.cpp"), "-o", exe], check=True)
    return exe


def test_golden_covers_the_edge_cases():
    meta, d = load_case("wrappers")
    assert d["term"].sum() >= 3 and d["trunc"].sum() >= 1
    assert np.any(np.abs(d["reward"]) == 10.0)            # reward clamp hit
    assert np.all(np.abs(d["obs"]) <= 10.0)
    assert np.count_nonzero(d["info_len"]) == d["term"].sum() + d["trunc"].sum() - np.sum(d["term"] * d["trunc"])


def test_oracle_wrappers_bit_exact_vs_golden():
    meta, d = load_case("wrappers")
    obs, out, mean, var = _oracle_run(meta["O"], meta["T"], meta["reset_at"], meta["gamma"])
    np.testing.assert_array_max_ulp(obs, d["obs"], maxulp=1)
    for k in ("reward", "term", "trunc", "info_ret", "info_len"):
        np.testing.assert_array_equal(out[k], d[k], err_msg=k)
    np.testing.assert_array_equal(mean, d["obs_mean_final"])
    np.testing.assert_array_equal(var, d["obs_var_final"])


def test_product_wrapper_chain_bit_exact_vs_golden(driver, tmp_path):
    meta, d = load_case("wrappers")
    Od, T = meta["O"], meta["T"]
    subprocess.run([driver, str(Od), str(T), str(meta["reset_at"]), str(tmp_path / "w.f32")], check=True)
    out = np.fromfile(tmp_path / "w.f32", dtype=np.float32)
    obs = out[:(T + 1) * Od].reshape(T + 1, Od)
    rest = out[(T + 1) * Od:].reshape(5, T)
    np.testing.assert_array_max_ulp(obs, d["obs"], maxulp=1)
    o_obs, _, _, _ = _oracle_run(Od, T, meta["reset_at"], meta["gamma"])
    np.testing.assert_array_equal(obs, o_obs)  # product == oracle (both IEEE sqrt), bit for bit
    for i, k in enumerate(("reward", "term", "trunc", "info_ret", "info_len")):
        np.testing.assert_array_equal(rest[i], d[k], err_msg=k)


def test_vector_oracle_chain_bit_exact_vs_golden():
    """orc_vwrap_* (one state per env behind a vector env — the checker of the device chain) fed the
    scripted env's raw stream reproduces the golden case in every env, bit for bit against the
    single-env oracle run."""
    meta, d = load_case("wrappers")
    Od, T = meta["O"], meta["T"]
    raw, r, te, tr, rs = O.wrappers_script(Od, T, meta["reset_at"])
    assert rs.sum() >= 4 and te.sum() >= 3
    E = 3
    w = O.VecWrappers(E, Od, meta["gamma"])
    obs0 = w.reset(np.tile(raw[0], (E, 1)))
    o_obs, o_out, o_mean, o_var = _oracle_run(Od, T, meta["reset_at"], meta["gamma"])
    np.testing.assert_array_equal(obs0, np.tile(o_obs[0], (E, 1)))
    for t in range(T):
        ob, rw = w.step(np.tile(raw[t + 1], (E, 1)), np.full(E, r[t], np.float32), np.full(E, te[t], np.float32),
                        np.full(E, rs[t], np.float32))
        np.testing.assert_array_equal(ob, np.tile(o_obs[t + 1], (E, 1)))
        np.testing.assert_array_equal(rw, np.full(E, o_out["reward"][t], np.float32))
        np.testing.assert_array_max_ulp(ob[0], d["obs"][t + 1], maxulp=1)
        np.testing.assert_array_equal(rw[0], d["reward"][t])
    st = w.state()
    np.testing.assert_array_equal(st["obs_mean"][1], d["obs_mean_final"])
    np.testing.assert_array_equal(st["obs_var"][2], d["obs_var_final"])
