"""The AC agent's fixed per-env-id observation normalisation (AgentImpl mean_ / std_;
ac_ppo_continuous_action.cpp Humanoid-v4 :496-497, Ant-v5 :521-522, Hopper-v5 :533-534,
HalfCheetah-v5 zeros / ones :510-511): the library's tables (ppo_obs_norm) equal the values the
reference writes (tests/golden/obs_norm.json, extracted by scripts/gen_obs_norm.py and converted to
float32 as torch::tensor({...}, kFloat) does), the initialiser packs them into mean_ / std_ of the
flat parameter vector, and they survive the LibTorch .pth round trip. Host-only calls (no GPU)."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libppo_hip.so not built")


def golden():
    with open(os.path.join(ROOT, "tests", "golden", "obs_norm.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("env_id,n", [("Humanoid-v4", 376), ("Ant-v5", 105), ("Hopper-v5", 11)])
def test_tables_match_reference_values(env_id, n):
    import ppo_amd
    m, s = ppo_amd.obs_norm(env_id)
    g = golden()[env_id]
    assert m.size == n and s.size == n
    np.testing.assert_array_equal(m, np.asarray(g["mean"], np.float32))
    np.testing.assert_array_equal(s, np.asarray(g["std"], np.float32))


def test_halfcheetah_is_identity_and_unknown_env_fails():
    import ppo_amd
    assert ppo_amd.obs_norm("HalfCheetah-v5") is None
    with pytest.raises(ppo_amd.PPOError, match="not implemented"):
        ppo_amd.obs_norm("Walker2d-v5")


@pytest.mark.parametrize("env_id", ["Ant-v5", "Hopper-v5", "Humanoid-v4"])
def test_packed_into_mean_std_and_pth_round_trip(env_id, tmp_path):
    import ppo_amd
    O_, A, lo, hi = ppo_amd.ENV_DIMS[env_id]
    L = ppo_amd.agent_layout(ppo_amd.PPO_NET_LN_BETA, O_, A, 256)
    p = ppo_amd.init_params(L, seed=1, env_id=env_id)
    m, s = ppo_amd.obs_norm(env_id)
    np.testing.assert_array_equal(p[L.omean:L.omean + O_], m)
    np.testing.assert_array_equal(p[L.ostd:L.ostd + O_], s)
    assert p[L.hi] == np.float32(hi) and p[L.lo] == np.float32(lo)
    path = str(tmp_path / "model.pth")
    ppo_amd.save_agent_pth(L, p, path)
    q = ppo_amd.load_agent_pth(L, path)
    np.testing.assert_array_equal(q, p)
