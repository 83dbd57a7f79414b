"""Pins the CPU oracle (oracle/ppo_oracle.c) against the reference-arithmetic golden vectors
(tests/golden/, produced by oracle/ref_harness.cpp which compiles the reference's rl_utils.h)."""
import numpy as np
import pytest

import oracle_lib as O
from golden_io import load_case


def rel(a, b):
    return np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(np.asarray(b, np.float64)), 1e-30)


@pytest.mark.parametrize("case,kind", [("ppo_act", 0), ("ac_act", 1)])
def test_layout_matches_named_parameters(case, kind):
    meta, _ = load_case(case)
    L = O.layout_init(kind, meta["O"], meta["A"], meta["H"])
    names = meta["params"]
    assert L.ntensors == len(names)
    for i, (name, n, grad) in enumerate(names):
        assert L.t_len[i] == n, name
        assert L.t_grad[i] == grad, name
    assert L.P == sum(n for _, n, _ in names)


def test_ppo_act_given_action():
    meta, d = load_case("ppo_act")
    L = O.layout_init(0, 17, 6, 64)
    _, lp, ent, v = O.get_action_and_value(L, d["params"], d["x"], 1, d["action"])
    np.testing.assert_allclose(lp, d["logprob"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(ent, d["entropy"], rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(v, d["value"], rtol=1e-5, atol=1e-6)
    mu, _, _, _ = O.get_action_and_value(L, d["params"], d["x"], 2)
    np.testing.assert_allclose(mu, d["mean"], rtol=1e-5, atol=1e-6)


def test_ac_act_given_and_mean():
    meta, d = load_case("ac_act")
    L = O.layout_init(1, 17, 6, 64)
    a, lp, ent, v = O.get_action_and_value(L, d["params"], d["x"], 1, d["action"])
    np.testing.assert_allclose(lp, d["logprob"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(ent, d["entropy"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(v, d["value"], rtol=1e-5, atol=1e-6)
    am, lpm, _, _ = O.get_action_and_value(L, d["params"], d["x"], 2)
    np.testing.assert_allclose(am, d["mean_action"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(lpm, d["mean_logprob"], rtol=1e-5, atol=2e-5)


def test_beta_distribution_spot_values():
    _, d = load_case("beta_dist")
    lib = O.lib()
    al, be, x = d["alpha"].astype(np.float64), d["beta"].astype(np.float64), d["x"].astype(np.float64)
    from math import lgamma, log
    lp = np.array([(a - 1) * log(xx) + (b - 1) * log(1 - xx) + lgamma(a + b) - lgamma(a) - lgamma(b)
                   for a, b, xx in zip(al, be, x)])
    ent = np.array([lgamma(a) + lgamma(b) - lgamma(a + b) - (2 - a - b) * lib.orc_digamma(a + b)
                    - (a - 1) * lib.orc_digamma(a) - (b - 1) * lib.orc_digamma(b) for a, b in zip(al, be)])
    np.testing.assert_allclose(lp, d["log_prob"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(ent, d["entropy"], rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("case,kind", [("ppo_update", 0), ("ac_update", 1)])
def test_minibatch_grad_clip_adam(case, kind):
    meta, d = load_case(case)
    L = O.layout_init(kind, meta["O"], meta["A"], meta["H"])
    cfg = O.LossCfg(meta["clip_coef"], meta["ent_coef"], meta["vf_coef"], meta["clip_vloss"], meta["norm_adv"])
    grad, stats = O.minibatch_grad(L, d["params"], d["x"], d["action"], d["old_logp"], d["adv"], d["ret"],
                                   d["old_v"], cfg)
    np.testing.assert_allclose(stats, d["stats"], rtol=2e-5, atol=2e-6)
    assert rel(grad, d["grad_raw"]) < 2e-5
    # per tensor too (small tensors must not hide in the global norm)
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            assert rel(grad[o:o + n], d["grad_raw"][o:o + n]) < 1e-4, t
    g, tn = O.clip_grad_norm(L, d["grad_raw"], meta["max_grad_norm"])
    assert abs(tn - d["total_norm"][0]) / d["total_norm"][0] < 1e-5
    assert rel(g, d["grad_clipped"]) < 1e-5
    p1, m, v = O.adam_step(L, d["params"], d["grad_clipped"], np.zeros(L.P), np.zeros(L.P), 1, meta["lr"],
                           meta["adam_eps"])
    np.testing.assert_allclose(p1, d["params_step1"], rtol=0, atol=2e-7)


def test_three_adam_steps_bias_correction():
    meta, d = load_case("ppo_update")
    L = O.layout_init(0, 17, 6, 64)
    cfg = O.LossCfg(meta["clip_coef"], meta["ent_coef"], meta["vf_coef"], meta["clip_vloss"], meta["norm_adv"])
    p = d["params"].copy(); m = np.zeros(L.P, np.float32); v = np.zeros(L.P, np.float32)
    for s in range(1, 4):
        g, _ = O.minibatch_grad(L, p, d["x"], d["action"], d["old_logp"], d["adv"], d["ret"], d["old_v"], cfg)
        g, _ = O.clip_grad_norm(L, g, meta["max_grad_norm"])
        p, m, v = O.adam_step(L, p, g, m, v, s, meta["lr"], meta["adam_eps"])
    np.testing.assert_allclose(p, d["params_step3"], rtol=0, atol=1e-6)
    assert rel(m, d["adam_m_step3"]) < 1e-4
    assert rel(v, d["adam_v_step3"]) < 1e-4


def test_distributed_equivalence_two_shards():
    """ac:830-849 + :877-885 — two shards with distributed adv stats + averaged grads."""
    meta, d = load_case("ac_update")
    L = O.layout_init(1, 17, 6, 64)
    cfg = O.LossCfg(meta["clip_coef"], meta["ent_coef"], meta["vf_coef"], meta["clip_vloss"], meta["norm_adv"])
    M, G = 64, 2
    Md = M // G
    adv = d["adv"].astype(np.float32)
    mean = np.float32(np.mean([adv[r * Md:(r + 1) * Md].astype(np.float64).mean() for r in range(G)]))
    ss = sum(float(np.sum((adv[r * Md:(r + 1) * Md].astype(np.float64) - mean) ** 2)) for r in range(G))
    std = np.float32(np.sqrt(ss / (G * Md - 1)))
    np.testing.assert_allclose([mean, std], d["dist2_adv_stats"], rtol=1e-6)
    gs = []
    for r in range(G):
        sl = slice(r * Md, (r + 1) * Md)
        g, _ = O.minibatch_grad(L, d["params"], d["x"][sl], d["action"][sl], d["old_logp"][sl], adv[sl],
                                d["ret"][sl], d["old_v"][sl], cfg, adv_mean=mean, adv_std=std)
        gs.append(g)
    gavg = (gs[0] + gs[1]) / 2
    assert rel(gavg, d["grad_dist2_avg"]) < 2e-5
    # ... and equals the single-shard gradient (data-parallel equivalence)
    assert rel(gavg, d["grad_raw"]) < 2e-5


def test_gae_bit_exact():
    meta, d = load_case("gae")
    adv, ret = O.gae(d["rewards"], d["values"], d["dones"], d["next_value"], d["next_done"], meta["gamma"],
                     meta["gae_lambda"])
    np.testing.assert_array_equal(adv, d["advantages"])
    np.testing.assert_array_equal(ret, d["returns"])
