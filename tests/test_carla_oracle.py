"""CaRL CNN agent: the C oracle's forward against the golden vectors of the
LibTorch replay of include/carla/carla_model.h (oracle/ref_harness.cpp, case carla_act), and the
flat layout against the reference's named_parameters() list recorded in the fixture."""
import numpy as np

import carla_inputs as CI
from golden_io import load_case


def test_layout_matches_named_parameters():
    meta, _ = load_case("carla_act")
    L = CI.layout()
    names = meta["params"]
    assert L.ntensors == len(names)
    assert L.P == meta["P"]
    for t, (name, n) in enumerate(names):
        assert L.t_len[t] == n, (t, name)
    assert [n for n, _ in names][:4] == ["action_space_high", "action_space_low", "cnn.0.weight", "cnn.0.bias"]


def test_oracle_forward_matches_golden():
    meta, d = load_case("carla_act")
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(meta["N"])
    o = CI.oracle_forward(L, p, bev, meas, vmeas, 2, act)
    np.testing.assert_allclose(o["features"], d["features"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(o["alpha"], d["alpha"], rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(o["beta"], d["beta"], rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(o["value"], d["value"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(o["logprob"], d["logprob"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(o["entropy"], d["entropy"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(o["action"], d["action_roundtrip"], rtol=1e-6, atol=1e-6)
    om = CI.oracle_forward(L, p, bev, meas, vmeas, 1)
    np.testing.assert_allclose(om["action"], d["mean_action"], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(om["logprob"], d["mean_logprob"], rtol=2e-5, atol=2e-5)
    orr = CI.oracle_forward(L, p, bev, meas, vmeas, 3)
    np.testing.assert_allclose(orr["action"], d["roach_action"], rtol=2e-5, atol=2e-6)
    np.testing.assert_allclose(orr["logprob"], d["roach_logprob"], rtol=2e-5, atol=2e-5)
