"""Host env stack (ppo.cpp_amd/gymcpp: SeqVectorEnv / ParVectorEnv + RecordEpisodeStatistics over
SyntheticCheetah) against the oracle's vector env, bit for bit — the same env the device rollout
uses (tests/test_gpu_parity.py::test_synth_env_bit_exact_vs_oracle), so host and device
collection see identical trajectories. Reference semantics: libs/gymcpp/gym.h:131-163 (clip,
next-step autoreset), libs/gymcpp/wrappers/common.h:11-66 (episode statistics)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("hostenv") / "host_env_driver")
    subprocess.run(["g++", "-O2", "-std=c++20", "-ffp-contract=off", "-pthread",
                    os.path.join(ROOT, "tests", "native", "host_env_driver.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("mode", ["seq", "par"])
def test_host_env_matches_oracle(driver, tmp_path, mode):
    E, T, A, Od, seed = 37, 1010, 6, 17, 5
    rng = np.random.default_rng(3)
    act = rng.uniform(-1.4, 1.4, (T, E, A)).astype(np.float32)
    act.tofile(tmp_path / "a.f32")
    subprocess.run([driver, mode, str(E), str(T), str(seed), str(tmp_path / "a.f32"), str(tmp_path / "o.f32")],
                   check=True)
    out = np.fromfile(tmp_path / "o.f32", dtype=np.float32)
    oenv = O.SynthEnv(E, Od, A)
    o0 = oenv.reset(seed)
    np.testing.assert_array_equal(out[:E * Od].reshape(E, Od), o0)
    per = E * Od + 5 * E
    base = E * Od
    finished = 0
    for t in range(T):
        blk = out[base + t * per: base + (t + 1) * per]
        o_obs, o_r, o_te, o_tr, o_ir, o_il = oenv.step(act[t])
        np.testing.assert_array_equal(blk[:E * Od].reshape(E, Od), o_obs)
        k = E * Od
        np.testing.assert_array_equal(blk[k:k + E], o_r)
        np.testing.assert_array_equal(blk[k + E:k + 2 * E], o_te)
        np.testing.assert_array_equal(blk[k + 2 * E:k + 3 * E], o_tr)
        np.testing.assert_array_equal(blk[k + 3 * E:k + 4 * E], o_ir)
        np.testing.assert_array_equal(blk[k + 4 * E:k + 5 * E], np.asarray(o_il, np.float32))
        finished += int((blk[k + 4 * E:k + 5 * E] > 0).sum())
    assert finished == E  # every env truncates once at step 1000, then autoresets
