"""The PPO update at the sizes the benchmarks run it, against the C oracle.

At the metric config (AC 2x256 LN/Beta, HalfCheetah O=17 / A=6, E=4096, T=128, 4 minibatches) each
minibatch is M = 131 072 rows, so every k_upd workgroup walks 16 row tiles and accumulates its slab
of small gradients across them, and k_dwf sums 128 split-K chunks; the cfg4 shard (Ant O=105 / A=8,
E=1024 per GPU) runs M = 32 768; cfg2 (PPO 2x64 tanh / Normal, Humanoid O=376 / A=17, E=1024,
T=2048, 32 minibatches) runs M = 65 536 through k_upd2 and k_dw2_dma. Here one update with one
minibatch of exactly that size (T x E with MB=1, EP=1 gives the same M, tiles per workgroup and
chunk count) is compared with the
oracle's gradient over the same gathered rows (oracle/ppo_oracle.c orc_minibatch_grad_part, row
chunks on a thread pool, partials added in a fixed order) and with the oracle's clip_grad_norm_ +
Adam step applied to the oracle's gradient.

Tolerances: raw gradient rel-L2 < 2e-4 overall and < 2e-3 per tensor, loss statistics rtol 2e-4
(the same bars as the M = 256 golden cases; MFMA fp32 accumulation order vs the oracle's double sums
is the only difference). Parameters after the Adam step:
  * against the oracle's clip_grad_norm_ + Adam applied to the GPU's own raw gradient: atol 2e-6
    (the clip and Adam arithmetic alone);
  * against the oracle's step of the oracle's gradient: atol 2e-6 + lr |dg| / (min |g| + eps) per
    element. Adam's first step moves every parameter by lr g / (|g| + eps), whose derivative in g is
    at most 1 / (|g| + eps): an element whose gradient is a near-cancelling sum over 131 072 rows
    (|g| ~ eps) turns the fp32-vs-double difference of that sum into an lr-sized difference of the
    step (measured: 30 of 146 225 elements beyond a flat 2e-6, at most 1.3e-5 = 0.05 lr).
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402
from test_gpu_parity import fill_storage, make_agent, random_params, rel  # noqa: E402


@pytest.mark.parametrize("name,kind,H,O_,A,E,T,clip,ent,lr,opts", [
    ("metric_halfcheetah", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, None),
    ("cfg4_shard_ant", 1, 256, 105, 8, 1024, 32, 0.1, 0.01, 2.5e-4, None),
    # the same two through k_upd32 (32x32x2 MFMA layout, create option upd_mfma=32)
    ("metric_halfcheetah_mfma32", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "upd_mfma=32"),
    ("cfg4_shard_ant_mfma32", 1, 256, 105, 8, 1024, 32, 0.1, 0.01, 2.5e-4, "upd_mfma=32"),
    ("metric_halfcheetah_mix", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "upd_mfma=mix"),
    # the default k_upd of these two runs its 256-wide GEMMs as split-bf16 piece products (upd_mfma=bx6);
    # the same two on fp32 16x16x4 MFMAs throughout (upd_mfma=16)
    ("metric_halfcheetah_f32", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "upd_mfma=16"),
    ("cfg4_shard_ant_f32", 1, 256, 105, 8, 1024, 32, 0.1, 0.01, 2.5e-4, "upd_mfma=16"),
    # the fused dW on exact bf16 piece products (k_dwf_bx, create option dw_mfma): all nine, and eight
    ("metric_halfcheetah_dw_bf16x9", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "dw_mfma=bf16x9"),
    ("metric_halfcheetah_dw_bf16x8", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "dw_mfma=bf16x8"),
    ("n8_shard_halfcheetah_dw_bf16x9", 1, 256, 17, 6, 512, 32, 0.1, 0.01, 2.5e-4, "dw_mfma=bf16x9"),
    # the minibatch as launch pairs of M / n rows (create option upd_split: k_upd + k_dwf per pair, the
    # pairs' slab and dW partial rows summed together), and a ragged last pair (127 968 = 3 x 32 000 +
    # 31 968 rows)
    ("metric_halfcheetah_split4", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "upd_split=4"),
    ("metric_halfcheetah_split2", 1, 256, 17, 6, 4096, 32, 0.1, 0.01, 2.5e-4, "upd_split=2"),
    ("ragged_split4", 1, 256, 17, 6, 3999, 32, 0.1, 0.01, 2.5e-4, "upd_split=4"),
    # cfg2: ppo_continuous_action Humanoid-v4, E=1024, T=2048, 32 minibatches -> M = 65 536 rows
    # (ppo:489-542; clip 0.2, ent_coef 0, lr 3e-4, ppo:60-67): k_upd2 walks 128 32-row tiles per
    # workgroup pair and k_dw2_dma sums 256 split-K chunks of 256 rows
    ("cfg2_humanoid", 0, 64, 376, 17, 1024, 64, 0.2, 0.0, 3e-4, None),
    # k_upd2's layer 1 on fp32 MFMAs (the default runs it as split-bf16 piece products, upd_mfma=bx6)
    ("cfg2_humanoid_f32", 0, 64, 376, 17, 1024, 64, 0.2, 0.0, 3e-4, "upd_mfma=16")])
def test_headline_minibatch_update_vs_oracle(name, kind, H, O_, A, E, T, clip, ent, lr, opts):
    M = E * T
    rng = np.random.default_rng(31)
    L = O.layout_init(kind, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (M, A)).astype(np.float32)
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    # old log-probs / values near the current policy's (the GPU's own forward with the given actions;
    # the comparison below is of the update only), so the clipped and unclipped branches both occur
    ag0 = make_agent(kind, O_, A, H, M)
    ag0.load_params(p)
    _, lp, _, v = ag0.get_action_and_value(DeviceArray.from_numpy(x), ppo_amd.PPO_GIVEN, DeviceArray.from_numpy(act))
    lp, v = lp.numpy(), v.numpy()
    ag0.close()
    olp = (lp + rng.standard_normal(M) * clip).astype(np.float32)
    ov = (v + rng.standard_normal(M) * 0.1).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    mgn, eps = 0.5, 1e-5

    ag = make_agent(kind, O_, A, H, E, T=T, MB=1, EP=1, clip=clip, ent=ent, max_grad_norm=mgn, adam_eps=eps,
                    options=opts)
    ag.load_params(p)
    fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
    st = ag.update(lr, perms=DeviceArray.from_numpy(perm), want_stats=True)
    g = ag.last_grad()
    p1 = ag.params()
    ag.close()

    cfg = O.LossCfg(clip, ent, 0.5, 1, 1)
    og, ost = O.minibatch_grad_parallel(L, p, x[perm], act[perm], olp[perm], adv[perm], ret[perm], ov[perm], cfg)
    assert rel(g, og) < 2e-4, rel(g, og)
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            assert rel(g[o:o + n], og[o:o + n]) < 2e-3, (t, rel(g[o:o + n], og[o:o + n]))
    np.testing.assert_allclose([st[k] for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl",
                                                 "clipfrac")], ost[:6], rtol=2e-4, atol=2e-6)
    assert 0.05 < ost[5] < 0.95  # both branches of the clipped surrogate are exercised
    gc, tn = O.clip_grad_norm(L, og, mgn)
    np.testing.assert_allclose(st["grad_norm"], tn, rtol=2e-4)
    zeros = np.zeros(L.P, np.float32)
    gg, _ = O.clip_grad_norm(L, g, mgn)
    pg_, _, _ = O.adam_step(L, p, gg, zeros, zeros, 1, lr, eps)
    np.testing.assert_allclose(p1, pg_, rtol=0, atol=2e-6)  # clip + Adam of the GPU's gradient
    op, _, _ = O.adam_step(L, p, gc, zeros, zeros, 1, lr, eps)
    g64, c64 = gg.astype(np.float64), gc.astype(np.float64)
    bound = 2e-6 + lr * np.abs(g64 - c64) / (np.minimum(np.abs(g64), np.abs(c64)) + eps)
    assert (np.abs(p1.astype(np.float64) - op) <= bound).all(), np.abs(p1 - op).max()
    assert np.mean(np.abs(p1 - op) > 2e-6) < 1e-3  # the sensitive elements are a small minority


@pytest.mark.parametrize("split", ["2", "3"])
def test_cfg2_split_update_matches_single_kernel(split):
    """cfg2's update in its split form (k_l1g: layer 1 of both trunks as one gathered GEMM into Z1,
    then k_upd2's tail at 2 / 3 workgroups per CU) against the single k_upd2 on fp32 MFMAs
    (upd2_split=0,upd_mfma=16) on the
    same minibatch (M = 16 384, ragged last tile: 16 383 rows): the layer-1 sums are the same products
    in another order (32x32x2 chains over k pairs instead of 16x16x4 chains), so gradients agree to
    fp32 accumulation noise (rel-L2 < 1e-5) and the loss statistics to rtol 1e-5."""
    kind, H, O_, A, E, T = 0, 64, 376, 17, 16383, 1
    M = E * T
    rng = np.random.default_rng(5)
    L = O.layout_init(kind, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = rng.standard_normal((M, A)).astype(np.float32) * 0.5
    olp = rng.standard_normal(M).astype(np.float32) - 20.0
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    ov = rng.standard_normal(M).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    out = []
    for opt in ("upd2_split=0,upd_mfma=16", f"upd2_split={split}"):
        ag = make_agent(kind, O_, A, H, E, T=T, MB=1, EP=1, clip=0.2, ent=0.0, options=opt)
        ag.load_params(p)
        fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
        st = ag.update(3e-4, perms=DeviceArray.from_numpy(perm), want_stats=True)
        out.append((ag.last_grad(), st, ag.params()))
        ag.close()
    (g0, s0, p0), (g1, s1, p1) = out
    assert rel(g1, g0) < 1e-5, rel(g1, g0)
    for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac", "grad_norm"):
        np.testing.assert_allclose(s1[k], s0[k], rtol=1e-5, atol=1e-7, err_msg=k)
    assert np.abs(p1 - p0).max() < 1e-5


@pytest.mark.parametrize("O_,A,E,opt32", [(17, 6, 999, "upd_mfma=32"), (105, 8, 777, "upd_mfma=32"),
                                          (16, 8, 333, "upd_mfma=32"), (17, 6, 999, "upd_mfma=mix")])
def test_upd32_matches_upd(O_, A, E, opt32):
    """k_upd32 (upd_mfma=32) against k_upd on the same minibatch, ragged last tile (E = M not a
    multiple of 32; O = 17: the one-column last k-block, 105: the synchronous wide gather, 16: one
    full k-block, A = 8: a full head tile): the same products summed in another order (32x32x2 chains and 32-lane reductions),
    so gradients agree to fp32 accumulation noise (rel-L2 < 2e-5) and the loss statistics to 2e-5."""
    kind, H, T = 1, 256, 1
    M = E * T
    rng = np.random.default_rng(11)
    L = O.layout_init(kind, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (M, A)).astype(np.float32)
    olp = rng.standard_normal(M).astype(np.float32)
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    ov = rng.standard_normal(M).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    out = []
    for opt in ("upd_mfma=16", opt32):
        ag = make_agent(kind, O_, A, H, E, T=T, MB=1, EP=1, clip=0.2, ent=0.01, options=opt)
        ag.load_params(p)
        fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
        st = ag.update(2.5e-4, perms=DeviceArray.from_numpy(perm), want_stats=True)
        out.append((ag.last_grad(), st))
        ag.close()
    (g0, s0), (g1, s1) = out
    assert rel(g1, g0) < 2e-5, rel(g1, g0)
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            assert rel(g1[o:o + n], g0[o:o + n]) < 2e-4, (t, rel(g1[o:o + n], g0[o:o + n]))
    for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac", "grad_norm"):
        np.testing.assert_allclose(s1[k], s0[k], rtol=2e-5, atol=1e-7, err_msg=k)


def test_upd32_refused_for_the_ppo_agent():
    with pytest.raises(ppo_amd.PPOError, match="upd_mfma=32"):
        make_agent(0, 17, 6, 64, 64, options="upd_mfma=32")


def test_refused_options_free_the_context():
    """A create refused for an option that cannot apply (upd_mfma=32 / upd2_split on the wrong agent)
    releases every device buffer it had allocated (the refusal paths used to `delete`
    the context after its stream and buffers existed). Device memory must not grow over repeated
    refusals at a metric-sized batch; rollout_kernel=valu on the PPO agent is refused up front."""
    import torch
    free0 = torch.cuda.mem_get_info(0)[0]
    for _ in range(6):
        with pytest.raises(ppo_amd.PPOError, match="upd_mfma=32"):
            make_agent(0, 17, 6, 64, 4096, T=128, MB=4, options="upd_mfma=32")
        with pytest.raises(ppo_amd.PPOError, match="upd2_split"):
            make_agent(1, 17, 6, 256, 4096, T=128, MB=4, options="upd2_split=2")
    free1 = torch.cuda.mem_get_info(0)[0]
    assert free0 - free1 < 64 << 20, (free0, free1)
    with pytest.raises(ppo_amd.PPOError, match="rollout_kernel=valu"):
        make_agent(0, 17, 6, 64, 64, options="rollout_kernel=valu")


@pytest.mark.parametrize("kind,O_,A,H,E,T", [(1, 17, 6, 256, 1024, 32), (1, 17, 6, 256, 1599, 8),
                                             (0, 376, 17, 64, 1024, 16), (0, 376, 17, 64, 1599, 8),
                                             (1, 105, 8, 256, 1024, 8)])
def test_split_bf16_dw_is_as_accurate_as_fp32_mfma(kind, O_, A, H, E, T):
    """k_dwf_bx (dW as exact bf16 piece products on v_mfma_f32_32x32x16_bf16, fp32 accumulation;
    opt-in create option dw_mfma=bf16x9 / bf16x8) against k_dwf_dma (v_mfma_f32_32x32x2_f32) on the
    same minibatch (M = 32 768 and a ragged 12 792): the dW1 / dW2 tensors of both trunks differ by
    accumulation rounding only (rel-L2 < 2e-6 between the two; measured <= 5.5e-7), bf16x9 and
    bf16x8 alike. Against the oracle's gradient (fp64 accumulation) the split form is measurably
    less exact than the fp32 MFMA on the well-conditioned tensors (critic dW2: 2.25e-7 against
    8.6e-8, the bf16 MFMA's internal accumulation) and equal where the k_upd hand-off dominates
    (actor: 2.4e-6 both): bar 4x the fp32 path's error + 1e-7. bf16x6 (k_upd's six products, the
    default dW since k_upd runs its split-bf16 form too: 17.3 -> 16.5 ms per metric iteration, DESIGN
    §8) measured 1.16e-7 against 7.7e-8 there. Every other gradient entry comes from k_upd / k_colsum
    and is bitwise the fp32 path's. The 64-wide agent (cfg2's Humanoid shape) runs the same three forms
    in k_dw2_dma (dW1 over the gathered 376-wide observation rows, dW2; one 16-row stage per
    32x32x16 bf16 MFMA k block), Ant's O = 105 (OP = 112) in the two-phase k_dw_dma the same way."""
    rng = np.random.default_rng(41)
    M = E * T
    L = O.layout_init(kind, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (M, A)).astype(np.float32)
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    olp = (rng.standard_normal(M) * 0.3 - 3.0).astype(np.float32)
    ov = (rng.standard_normal(M) * 0.1).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    grads = {}
    for opt in ("f32", "bf16x9", "bf16x8", "bf16x6"):
        ag = make_agent(kind, O_, A, H, E, T=T, MB=1, EP=1, clip=0.1, options=f"dw_mfma={opt}")
        ag.load_params(p)
        fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
        ag.update(2.5e-4, perms=DeviceArray.from_numpy(perm), want_stats=False)
        grads[opt] = ag.last_grad()
        ag.close()
    cfg = O.LossCfg(0.1, 0.01, 0.5, 1, 1)
    og, _ = O.minibatch_grad_parallel(L, p, x[perm], act[perm], olp[perm], adv[perm], ret[perm], ov[perm], cfg)
    dw = set()
    for tr in (L.critic, L.actor):
        dw.update((tr[0], tr[4]))  # W1, W2 offsets
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        g32 = grads["f32"][o:o + n]
        for opt in ("bf16x9", "bf16x8", "bf16x6"):
            gb = grads[opt][o:o + n]
            if o not in dw:
                np.testing.assert_array_equal(gb, g32, err_msg=f"tensor {t} {opt}")
                continue
            assert rel(gb, g32) < 2e-6, (t, opt, rel(gb, g32))
            e32, eb = rel(g32, og[o:o + n]), rel(gb, og[o:o + n])
            print(f"tensor {t} ({n}): {opt} vs f32 {rel(gb, g32):.2e}; vs oracle f32 {e32:.2e} {opt} {eb:.2e}")
            assert eb <= 4.0 * e32 + 1e-7, (t, opt, e32, eb)


@pytest.mark.parametrize("O_,A,E", [(17, 6, 999), (105, 8, 777), (16, 8, 333), (17, 6, 4096)])
def test_upd_bx6_is_as_accurate_as_fp32_mfma(O_, A, E):
    """k_upd's split-bf16 form (upd_mfma=bx6: layer 2 and dh1 = W2^T dz2 as six bf16 piece products
    per fp32 product on v_mfma_f32_16x16x32_bf16, fp32 accumulation) against the fp32-MFMA k_upd on
    the same minibatch (ragged last tiles; O = 17 / 105 (the synchronous wide gather) / 16; A = 8: a full head tile) and both
    against the oracle's gradient (fp64 accumulation). The dropped piece products are below 2^-23 of
    each product, so the split form must be as close to the oracle as the fp32 MFMA form: per
    gradient tensor within 1.5x its error + 1e-6 (a few ulps: one-element tensors), and within 2e-5 rel-L2 of it overall; loss
    statistics rtol 2e-5."""
    kind, H, T = 1, 256, 1
    M = E * T
    rng = np.random.default_rng(13)
    L = O.layout_init(kind, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (M, A)).astype(np.float32)
    olp = (rng.standard_normal(M) * 0.3 - 3.0).astype(np.float32)
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    ov = (rng.standard_normal(M) * 0.1).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    out = {}
    for opt in ("upd_mfma=16", "upd_mfma=bx6"):
        ag = make_agent(kind, O_, A, H, E, T=T, MB=1, EP=1, clip=0.2, ent=0.01, options=opt)
        ag.load_params(p)
        fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
        st = ag.update(2.5e-4, perms=DeviceArray.from_numpy(perm), want_stats=True)
        out[opt] = (ag.last_grad(), st, ag.params())
        ag.close()
    (g0, s0, p0), (g1, s1, p1) = out["upd_mfma=16"], out["upd_mfma=bx6"]
    cfg = O.LossCfg(0.2, 0.01, 0.5, 1, 1)
    og, _ = O.minibatch_grad_parallel(L, p, x[perm], act[perm], olp[perm], adv[perm], ret[perm], ov[perm], cfg)
    print(f"\nbx6 vs f32 {rel(g1, g0):.2e}; vs oracle: f32 {rel(g0, og):.2e} bx6 {rel(g1, og):.2e}")
    assert rel(g1, g0) < 2e-5, rel(g1, g0)
    worst = 0.0
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            e0, e1 = rel(g0[o:o + n], og[o:o + n]), rel(g1[o:o + n], og[o:o + n])
            worst = max(worst, e1 / max(e0, 1e-12))
            print(f"  tensor {t:2d} ({n:6d}): f32 {e0:.2e} bx6 {e1:.2e}")
            assert e1 <= 1.5 * e0 + 1e-6, (t, e0, e1)
    print(f"worst per-tensor error ratio bx6 / f32: {worst:.2f}")
    for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac", "grad_norm"):
        np.testing.assert_allclose(s1[k], s0[k], rtol=2e-5, atol=1e-7, err_msg=k)
    assert np.abs(p1 - p0).max() < 1e-5


def test_upd_bx6_refused_where_it_does_not_apply():
    with pytest.raises(ppo_amd.PPOError, match="upd_mfma=bx6"):
        make_agent(0, 17, 6, 64, 64, options="upd_mfma=bx6")  # the 64-wide agent off cfg2's shape
    with pytest.raises(ppo_amd.PPOError, match="upd_mfma=bx6"):
        make_agent(1, 376, 17, 256, 64, options="upd_mfma=bx6")  # 34 heads: three head tiles


@pytest.mark.parametrize("E,T", [(2047, 1), (1024, 16)])
def test_upd2_bx6_is_as_accurate_as_fp32_mfma(E, T):
    """k_upd2 with layer 1 (K = OP = 384) as split-bf16 piece products (upd_mfma=bx6, the default at
    cfg2's Humanoid shape: each staged chunk split once into bf16 pieces) against its fp32-MFMA form
    (upd_mfma=16) and both against the oracle's gradient (fp64 accumulation), M = 2 047 (ragged last
    tile) and 16 384: per gradient tensor within 1.5x the fp32 form's error + 1e-6, overall within
    2e-5 rel-L2 of it; loss statistics rtol 2e-5."""
    kind, H, O_, A = 0, 64, 376, 17
    M = E * T
    rng = np.random.default_rng(17)
    L = O.layout_init(kind, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = (rng.standard_normal((M, A)) * 0.5).astype(np.float32)
    olp = (rng.standard_normal(M) * 0.3 - 20.0).astype(np.float32)
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    ov = rng.standard_normal(M).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    out = {}
    for opt in ("upd_mfma=16", "upd_mfma=bx6"):
        ag = make_agent(kind, O_, A, H, E, T=T, MB=1, EP=1, clip=0.2, ent=0.0, options=opt)
        assert ag.kernel_info().startswith("update=k_upd2/" + ("f32" if opt.endswith("16") else "bx6"))
        ag.load_params(p)
        fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
        st = ag.update(3e-4, perms=DeviceArray.from_numpy(perm), want_stats=True)
        out[opt] = (ag.last_grad(), st)
        ag.close()
    (g0, s0), (g1, s1) = out["upd_mfma=16"], out["upd_mfma=bx6"]
    cfg = O.LossCfg(0.2, 0.0, 0.5, 1, 1)
    og, _ = O.minibatch_grad_parallel(L, p, x[perm], act[perm], olp[perm], adv[perm], ret[perm], ov[perm], cfg)
    print(f"\nbx6 vs f32 {rel(g1, g0):.2e}; vs oracle: f32 {rel(g0, og):.2e} bx6 {rel(g1, og):.2e}")
    assert rel(g1, g0) < 2e-5, rel(g1, g0)
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            e0, e1 = rel(g0[o:o + n], og[o:o + n]), rel(g1[o:o + n], og[o:o + n])
            assert e1 <= 1.5 * e0 + 1e-6, (t, e0, e1)
    for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac", "grad_norm"):
        np.testing.assert_allclose(s1[k], s0[k], rtol=2e-5, atol=1e-7, err_msg=k)


@pytest.mark.parametrize("E,T,O_", [(4096, 32, 17), (3999, 4, 17), (512, 32, 16), (700, 9, 11), (1024, 8, 20)])
def test_h1_recompute_is_bitwise_the_stored_h1(E, T, O_):
    """h1_handoff=recompute (the default where it applies): k_upd writes each row's layer-1 LayerNorm
    statistics (8 bytes) instead of its 1 KB H1 row, and k_dwf_bx recomputes H1 per 16-row stage from
    the staged Xn rows with k_upd's own layer-1 chain (W1 swizzled copy, bias init, the same 16x16x4 fp32
    MFMA k order and last-block k-steps, the same LayerNorm affine + ReLU expression). Against
    h1_handoff=store on the same minibatch: gradient, stepped parameters and loss statistics bitwise
    equal — at the metric minibatch (M = 131 072: 128 chunks, one output slice), ragged (M = 15 996),
    the small-minibatch geometry (two output slices) and the other layer-1 shapes (OP = 16 / 32, one or
    four k-steps in the last k block)."""
    M = E * T
    rng = np.random.default_rng(43)
    A, H = 6, 256
    L = O.layout_init(1, O_, A, H)
    p = random_params(L, rng)
    x = rng.standard_normal((M, O_)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (M, A)).astype(np.float32)
    olp = (rng.standard_normal(M) * 0.3 - 3.0).astype(np.float32)
    adv = rng.standard_normal(M).astype(np.float32)
    ret = rng.standard_normal(M).astype(np.float32)
    ov = rng.standard_normal(M).astype(np.float32)
    perm = rng.permutation(M).astype(np.int32)
    out = []
    for opt in ("h1_handoff=store", "h1_handoff=recompute"):
        ag = make_agent(1, O_, A, H, E, T=T, MB=1, EP=1, clip=0.2, ent=0.01, options=opt)
        try:
            assert ("h1rc" in ag.kernel_info()) == opt.endswith("recompute"), ag.kernel_info()
            ag.load_params(p)
            fill_storage(ag, T, E, x, act, olp, adv, ret, ov)
            st = ag.update(2.5e-4, perms=DeviceArray.from_numpy(perm), want_stats=True)
            out.append((ag.last_grad(), ag.params(), st))
        finally:
            ag.close()
    (g0, p0, s0), (g1, p1, s1) = out
    np.testing.assert_array_equal(g1, g0)
    np.testing.assert_array_equal(p1, p0)
    assert s0 == s1
