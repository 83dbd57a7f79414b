"""CaRL CNN agent: the C oracle's forward against the golden vectors of the
LibTorch replay of include/carla/carla_model.h (oracle/ref_harness.cpp, case carla_act), and the
flat layout against the reference's named_parameters() list recorded in the fixture."""
import numpy as np
import pytest

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


def _summary(L, flat, idx):
    """per tensor: sum, sum of squares, the entries at the golden's sample indices"""
    rows = []
    for t in range(L.ntensors):
        x = flat[L.t_off[t]:L.t_off[t] + L.t_len[t]].astype(np.float64)
        rows.append(np.concatenate([[x.sum(), (x * x).sum()], x[idx[t]]]))
    return np.array(rows)


def assert_rows_close(a, b, rtol, atol_rows):
    """|a - b| <= rtol |b| + atol_rows[row] elementwise (atol scaled per tensor)"""
    err = np.abs(a - b) - (rtol * np.abs(b) + atol_rows)
    bad = np.argwhere(err > 0)
    assert bad.size == 0, f"{len(bad)} entries off, worst row/col {np.unravel_index(err.argmax(), err.shape)}: " \
                          f"{a[np.unravel_index(err.argmax(), err.shape)]} vs {b[np.unravel_index(err.argmax(), err.shape)]}"


def test_torch_reference_update_matches_golden():
    """tests/carla_torch_ref.py (the fp32 reference the GPU update is checked against in full) equals
    the LibTorch replay of ac_ppo_carla.cpp:540-619 on the carla_update case."""
    torch = pytest.importorskip("torch")
    import carla_torch_ref as TR
    torch.set_num_threads(4)
    meta, g = load_case("carla_update")
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(meta["N"])
    grad, stats, total, newp, lp, val = TR.update(L, p, bev, meas, vmeas, act, g["old_logp"], g["adv"], g["ret"],
                                                  g["old_v"], clip=meta["clip_coef"], ent_coef=meta["ent_coef"],
                                                  vf_coef=meta["vf_coef"], max_grad_norm=meta["max_grad_norm"],
                                                  lr=meta["lr"], eps=meta["adam_eps"])
    np.testing.assert_allclose(lp, g["logprob"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(val, g["value"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(stats, g["stats"][:6], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(total, g["total_norm"][0], rtol=1e-5)
    gs = _summary(L, grad, g["sample_idx"])
    scale = np.sqrt(g["grad_summary"][:, 1:2] / np.array([[max(L.t_len[t], 1)] for t in range(L.ntensors)]))
    assert_rows_close(gs[:, 2:], g["grad_summary"][:, 2:], 1e-3, 1e-4 * scale + 1e-9)
    np.testing.assert_allclose(gs[:, 1], g["grad_summary"][:, 1], rtol=1e-4, atol=1e-12)
    ps = _summary(L, newp, g["sample_idx"])
    np.testing.assert_allclose(ps[:, 2:], g["param_step1_summary"][:, 2:], rtol=0, atol=2e-6)
