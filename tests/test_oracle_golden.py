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


# ------------------------------------------------------------------------------------------------
# round-2 cases at the reference's real widths (AC 2x256 LayerNorm trunks at HalfCheetah and Ant
# dims, ac:159-186; PPO 2x64 tanh at Humanoid O=376 / A=17, ppo:122-139), ragged and long GAE
# ------------------------------------------------------------------------------------------------
from golden_inputs import column_fnv, gae_long_inputs, hash_params  # noqa: E402

WIDTH_CASES = [("ac256", 1), ("ant256", 1), ("hum376", 0)]


def width_params(pre):
    meta, _ = load_case(pre + "_act")
    L = O.layout_init(meta["kind"], meta["O"], meta["A"], meta["H"])
    return meta, L, hash_params(L, meta["hash_base"], meta.get("hi", 1.0), meta.get("lo", -1.0))


def ac_adv_stats(adv, G=1):
    """ac:830-849: mean averaged over G row shards, sum of squares summed, Bessel over G*M_dev."""
    adv = np.asarray(adv, np.float32)
    Md = adv.size // G
    mean = np.float32(np.mean([adv[r * Md:(r + 1) * Md].astype(np.float64).mean() for r in range(G)]))
    ss = sum(float(np.sum((adv[r * Md:(r + 1) * Md].astype(np.float64) - mean) ** 2)) for r in range(G))
    return mean, np.float32(np.sqrt(ss / (G * Md - 1)))


@pytest.mark.parametrize("pre,kind", WIDTH_CASES)
def test_width_layout_matches_named_parameters(pre, kind):
    meta, L, p = width_params(pre)
    names = meta["params"]
    assert L.ntensors == len(names) and L.P == sum(n for _, n, _ in names)
    for i, (name, n, grad) in enumerate(names):
        assert L.t_len[i] == n and L.t_grad[i] == grad, name


@pytest.mark.parametrize("pre,kind", WIDTH_CASES)
def test_width_act_vs_golden(pre, kind):
    meta, L, p = width_params(pre)
    _, d = load_case(pre + "_act")
    _, lp, ent, v = O.get_action_and_value(L, p, d["x"], 1, d["action"])
    np.testing.assert_allclose(lp, d["logprob"], rtol=1e-5, atol=5e-5)
    np.testing.assert_allclose(ent, d["entropy"], rtol=1e-5, atol=5e-5)
    np.testing.assert_allclose(v, d["value"], rtol=1e-5, atol=1e-5)
    am, lpm, _, _ = O.get_action_and_value(L, p, d["x"], 2)
    if kind == 1:
        np.testing.assert_allclose(am, d["mean_action"], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(lpm, d["mean_logprob"], rtol=1e-5, atol=5e-5)
    else:
        np.testing.assert_allclose(am, d["mean"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("pre,kind", WIDTH_CASES)
def test_width_update_vs_golden(pre, kind):
    """grad, stats, clip norm, 1 and 3 Adam steps; AC uses the trainer's distributed-form advantage
    statistics with world_size = 1 (ac:830-849), PPO Tensor::std() (ppo:511)."""
    meta, L, p = width_params(pre)
    mu, du = load_case(pre + "_update")
    cfg = O.LossCfg(mu["clip_coef"], mu["ent_coef"], mu["vf_coef"], mu["clip_vloss"], mu["norm_adv"])
    am, asd = ac_adv_stats(du["adv"]) if kind == 1 else O.adv_stats(du["adv"])
    args = (du["x"], du["action"], du["old_logp"], du["adv"], du["ret"], du["old_v"])
    grad, stats = O.minibatch_grad(L, p, *args, cfg, adv_mean=am, adv_std=asd)
    np.testing.assert_allclose(stats[:6], du["stats"][:6], rtol=5e-5, atol=5e-6)
    assert rel(grad, du["grad_raw"]) < 2e-5
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            assert rel(grad[o:o + n], du["grad_raw"][o:o + n]) < 2e-4, t
    m = np.zeros(L.P, np.float32); v = np.zeros(L.P, np.float32)
    for s in range(1, 4):
        if s > 1:
            grad, _ = O.minibatch_grad(L, p, *args, cfg, adv_mean=am, adv_std=asd)
        g, tn = O.clip_grad_norm(L, grad, mu["max_grad_norm"])
        if s == 1:
            assert abs(tn - du["total_norm"][0]) / du["total_norm"][0] < 2e-5
        p, m, v = O.adam_step(L, p, g, m, v, s, mu["lr"], mu["adam_eps"])
        if s == 1:
            np.testing.assert_allclose(p, du["params_step1"], rtol=0, atol=5e-7)
    np.testing.assert_allclose(p, du["params_step3"], rtol=0, atol=2e-6)


@pytest.mark.parametrize("pre", ["ac256", "ant256"])
def test_width_distributed_two_shards(pre):
    meta, L, p = width_params(pre)
    mu, d = load_case(pre + "_update")
    cfg = O.LossCfg(mu["clip_coef"], mu["ent_coef"], mu["vf_coef"], mu["clip_vloss"], mu["norm_adv"])
    mean, std = ac_adv_stats(d["adv"], G=2)
    np.testing.assert_allclose([mean, std], d["dist2_adv_stats"], rtol=1e-6)
    Md = d["adv"].size // 2
    gs = []
    for r in range(2):
        sl = slice(r * Md, (r + 1) * Md)
        g, _ = O.minibatch_grad(L, p, d["x"][sl], d["action"][sl], d["old_logp"][sl], d["adv"][sl], d["ret"][sl],
                                d["old_v"][sl], cfg, adv_mean=mean, adv_std=std)
        gs.append(g)
    assert rel((gs[0] + gs[1]) / 2, d["grad_dist2_avg"]) < 2e-5


@pytest.mark.parametrize("T", [1, 7, 33])
def test_gae_ragged_bit_exact(T):
    meta, d = load_case(f"gae_t{T}")
    adv, ret = O.gae(d["rewards"], d["values"], d["dones"], d["next_value"], d["next_done"], 0.99, 0.95)
    np.testing.assert_array_equal(adv, d["advantages"])
    np.testing.assert_array_equal(ret, d["returns"])


def test_gae_long_bit_exact():
    """cfg2's T=2048 (E=1024): inputs regenerated from the hash streams, outputs via column hashes."""
    meta, d = load_case("gae_long")
    r, v, dn, nv, nd = gae_long_inputs(meta["T"], meta["E"])
    adv, ret = O.gae(r, v, dn, nv, nd, 0.99, 0.95)
    np.testing.assert_array_equal(adv[:, :8], d["adv_cols8"])
    np.testing.assert_array_equal(column_fnv(adv), d["adv_fnv"])
    np.testing.assert_array_equal(column_fnv(ret), d["ret_fnv"])


# ------------------------------------------------------------------------------------------------
# end-to-end fixture (e2e_ppo / e2e_ac): the oracle runs the trainer loop with the same contract
# ------------------------------------------------------------------------------------------------
def oracle_trainer(case, iterations):
    """Oracle restatement of ppo_amd.Trainer (lr anneal, Philox rollout on the oracle env, GAE,
    Feistel-permuted minibatch updates) for the golden e2e case's config; returns per-iteration
    (pg, v, ent, okl, kl, episodic return sum, episodes) rows and the final parameters."""
    meta, d = load_case(case)
    kind, E, T, MB, EP = meta["kind"], meta["E"], meta["T"], meta["MB"], meta["EP"]
    L = O.layout_init(kind, 17, 6, 64 if kind == 0 else 256)
    p = hash_params(L, meta["hash_base"])
    m = np.zeros(L.P, np.float32); v = np.zeros(L.P, np.float32); step = 0
    env = O.SynthEnv(E, 17, 6, wrappers=meta.get("wrappers", False))
    nobs = env.reset(1); ndone = np.zeros(E, np.float32)
    cfg = O.LossCfg(meta["clip_coef"], meta["ent_coef"], 0.5, 1, 1)
    rows = []
    for it in range(iterations):
        lr = float(np.float32(np.float32(1) - np.float32(it) / np.float32(meta["iterations"])) * np.float32(meta["lr"]))
        bo = np.zeros((T, E, 17), np.float32); ba = np.zeros((T, E, 6), np.float32)
        bl, br, bd, bv = (np.zeros((T, E), np.float32) for _ in range(4))
        rs, ne = 0.0, 0
        for t in range(T):
            bo[t] = nobs; bd[t] = ndone
            a, lp, _, val = O.get_action_and_value(L, p, nobs, 0, seed=1, rank=0, env_base=0, step_id=it * T + t)
            ba[t] = a; bl[t] = lp; bv[t] = val
            nobs, r, te, tr, ir, il = env.step(a)
            br[t] = r; ndone = np.maximum(te, tr)
            rs += float(ir[il > 0].sum()); ne += int((il > 0).sum())
        _, _, _, nv = O.get_action_and_value(L, p, nobs, 2)
        adv, ret = O.gae(br, bv, bd, nv, ndone, 0.99, 0.95)
        p, m, v, step, st = O.update(L, p, m, v, step, bo.reshape(-1, 17), ba.reshape(-1, 6), bl.reshape(-1),
                                     adv.reshape(-1), ret.reshape(-1), bv.reshape(-1), EP, MB, lr, 0.5, 1e-5, cfg,
                                     seed=1, rank=0, epoch_counter0=it * EP)
        rows.append(list(st[:5]) + [rs, ne])
    return np.array(rows, np.float64), p, d


def test_e2e_oracle_ppo_matches_libtorch_replay():
    rows, p, d = oracle_trainer("e2e_ppo", 8)
    want = d["stats"].astype(np.float64)
    np.testing.assert_allclose(rows[:, :5], want[:, :5], rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(rows[:, 5:], want[:, 6:], rtol=1e-5)
    np.testing.assert_allclose(p, d["params_final"], rtol=0, atol=1e-6)


def test_e2e_oracle_ppo_wrapped_matches_libtorch_replay():
    """The PPO trainer loop with the ppo:41-49 wrapper chain on every env (e2e_ppo_wrapped): the
    oracle (IEEE sqrtf in NormalizeObservation) against the LibTorch replay (MKL's vsSqrt, 1 ulp low
    on ~0.65 % of inputs, test_wrappers.py) — the stated bars of the GPU test."""
    rows, p, d = oracle_trainer("e2e_ppo_wrapped", 8)
    want = d["stats"].astype(np.float64)
    print("\nmax rel diff per column:", (np.abs(rows[:, :5] - want[:, :5]) / np.abs(want[:, :5])).max(0),
          "params max abs diff", np.abs(p - d["params_final"]).max())
    np.testing.assert_array_equal(rows[:, 6], want[:, 7])
    np.testing.assert_allclose(rows[:, :3], want[:, :3], rtol=2e-4, atol=1e-6)
    np.testing.assert_allclose(rows[:, 3:5], want[:, 3:5], rtol=0, atol=1e-5)
    np.testing.assert_allclose(rows[:, 5], want[:, 6], rtol=1e-5)
    np.testing.assert_allclose(p, d["params_final"], rtol=0, atol=1e-5)


def test_e2e_oracle_vs_libtorch_drift():
    """The AC agent's training dynamics amplify ulp-level differences: the oracle (double
    accumulators) and the LibTorch replay agree to ~1e-6 for two iterations and then drift apart
    (no sampling flips; this is the optimizer amplifying fp32 noise) — the reason the GPU e2e test
    states a looser tolerance for later AC iterations."""
    rows, _, d = oracle_trainer("e2e_ac", 3)
    want = d["stats"].astype(np.float64)[:3]
    np.testing.assert_allclose(rows[:2, :3], want[:2, :3], rtol=2e-5, atol=2e-6)
    drift = np.abs(rows[2, :3] - want[2, :3]) / np.abs(want[2, :3])
    assert drift.max() < 5e-2


def test_parallel_minibatch_grad_equals_serial():
    """The thread-pool form used at the headline minibatch size (test_gpu_update_headline) equals the
    serial oracle: disjoint row ranges, partials added in double in a fixed order."""
    L = O.layout_init(1, 17, 6, 256)
    rng = np.random.default_rng(3)
    p = (rng.standard_normal(L.P) * 0.05).astype(np.float32)
    p[L.hi], p[L.lo] = 1.0, -1.0
    p[L.ostd:L.ostd + 17] = 1.0
    M = 1500
    x = rng.standard_normal((M, 17)).astype(np.float32)
    a = rng.uniform(-0.9, 0.9, (M, 6)).astype(np.float32)
    z = [rng.standard_normal(M).astype(np.float32) for _ in range(4)]
    cfg = O.LossCfg(0.1, 0.01, 0.5, 1, 1)
    g1, s1 = O.minibatch_grad(L, p, x, a, *z, cfg)
    g2, s2 = O.minibatch_grad_parallel(L, p, x, a, *z, cfg, threads=4, chunk=256)
    np.testing.assert_allclose(g2, g1, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(s2, s1, rtol=1e-6, atol=1e-9)
