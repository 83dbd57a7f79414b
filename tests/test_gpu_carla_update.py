"""GPU parity of the CaRL PPO minibatch update (ppo_carla_update: loss, backward through heads, MLPs
and the six convolutions, clip_grad_norm_, Adam; ac_ppo_carla.cpp:540-619) through the C-ABI.

References: the LibTorch replay of the reference module (golden case carla_update: stats, total
norm, per-tensor gradient and stepped-parameter summaries) and tests/carla_torch_ref.py, a plain
PyTorch fp32 reference pinned to that golden (test_carla_oracle), for the full gradient vector.
Tolerances: the gradient is an fp32 MFMA chain in a different summation order from PyTorch's
(reductions over up to n * 8836 pixels) — per-tensor relative L2 error < 1e-3 and element-wise
|d| <= 2e-3 |ref| + 1e-3 * rms(tensor); stats rtol 1e-4; total norm rtol 1e-4; parameters after
one Adam step atol 2e-6 (the step is lr-sized, 3e-4)."""
import numpy as np
import pytest

import carla_inputs as CI
from golden_io import load_case

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402

import carla_torch_ref as TR  # noqa: E402

CFG = dict(clip=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, lr=3e-4, eps=1e-5)


def _run_update(ag, bev, meas, vmeas, act, old_logp, adv, ret, old_v):
    d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                   for x in (meas, vmeas, act, old_logp, adv, ret, old_v)]
    st = ag.update(*d, lr=CFG["lr"], clip_coef=CFG["clip"], ent_coef=CFG["ent_coef"], vf_coef=CFG["vf_coef"],
                   max_grad_norm=CFG["max_grad_norm"], adam_eps=CFG["eps"])
    return st, ag.last_grad(), ag.params()


def _check_grad(L, got, ref):
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        g, r = got[o:o + n].astype(np.float64), ref[o:o + n].astype(np.float64)
        nr = np.linalg.norm(r)
        if nr == 0:
            assert np.abs(g).max() == 0, t
            continue
        assert np.linalg.norm(g - r) / nr < 1e-3, (t, np.linalg.norm(g - r) / nr)
        rms = nr / np.sqrt(n)
        assert (np.abs(g - r) <= 2e-3 * np.abs(r) + 1e-3 * rms).all(), t


@pytest.fixture(scope="module")
def agent():
    ppo_amd.set_device(0)
    ag = ppo_amd.CarlaAgent(max_batch=32, seed=7)
    yield ag
    ag.close()


def test_update_vs_golden_and_torch(agent):
    torch.set_num_threads(8)
    meta, g = load_case("carla_update")
    L = CI.layout()
    p = CI.params(L)
    agent.load_params(p)
    agent.load_adam(np.zeros(L.P, np.float32), np.zeros(L.P, np.float32), 0)
    bev, meas, vmeas, act = CI.inputs(meta["N"])
    st, grad, newp = _run_update(agent, bev, meas, vmeas, act, g["old_logp"], g["adv"], g["ret"], g["old_v"])
    ref_g, ref_st, ref_total, ref_p, _, _ = TR.update(L, p, bev, meas, vmeas, act, g["old_logp"], g["adv"], g["ret"],
                                                      g["old_v"], **CFG)
    stats = np.array([st[k] for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac")])
    np.testing.assert_allclose(stats, g["stats"][:6], rtol=1e-4, atol=2e-6)
    np.testing.assert_allclose(st["grad_norm"], g["total_norm"][0], rtol=1e-4)
    _check_grad(L, grad, ref_g)
    # golden summaries (LibTorch itself): per-tensor sums of squares and sampled entries
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        x = grad[o:o + n].astype(np.float64)
        gs = g["grad_summary"][t]
        np.testing.assert_allclose((x * x).sum(), gs[1], rtol=2e-3, atol=1e-12)
        rms = np.sqrt(gs[1] / n)
        assert (np.abs(x[g["sample_idx"][t]] - gs[2:]) <= 2e-3 * np.abs(gs[2:]) + 1e-3 * rms + 1e-12).all(), t
        pp = newp[o:o + n][g["sample_idx"][t]]
        np.testing.assert_allclose(pp, g["param_step1_summary"][t][2:], rtol=0, atol=2e-6)
    np.testing.assert_allclose(newp, ref_p, rtol=0, atol=2e-6)
    m, v, step = agent.adam_state()
    assert step == 1 and np.isfinite(m).all() and (v >= 0).all()
    assert m[0] == 0 and m[1] == 0  # action_space_high / _low carry no optimizer state


def test_update_larger_batch_vs_torch(agent):
    """n = 32 rows: several wgrad chunks per layer and a ragged last chunk; two consecutive steps."""
    torch.set_num_threads(8)
    L = CI.layout()
    p = CI.params(L)
    agent.load_params(p)
    agent.load_adam(np.zeros(L.P, np.float32), np.zeros(L.P, np.float32), 0)
    n = 32
    rng = np.random.default_rng(5)
    bev = rng.integers(0, 256, size=(n, 15, 192, 192), dtype=np.uint8)
    meas = rng.uniform(-1, 1, (n, 8)).astype(np.float32)
    vmeas = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (n, 2)).astype(np.float32)
    adv = rng.standard_normal(n).astype(np.float32)
    ret = rng.standard_normal(n).astype(np.float32)
    old_v = rng.standard_normal(n).astype(np.float32) * 0.1
    old_logp = rng.standard_normal(n).astype(np.float32) * 0.2
    st, grad, newp = _run_update(agent, bev, meas, vmeas, act, old_logp, adv, ret, old_v)
    ref_g, ref_st, ref_total, ref_p, _, _ = TR.update(L, p, bev, meas, vmeas, act, old_logp, adv, ret, old_v, **CFG)
    _check_grad(L, grad, ref_g)
    np.testing.assert_allclose(st["grad_norm"], ref_total, rtol=1e-4)
    np.testing.assert_allclose(newp, ref_p, rtol=0, atol=2e-6)
    st2, grad2, newp2 = _run_update(agent, bev, meas, vmeas, act, old_logp, adv, ret, old_v)
    assert np.isfinite(newp2).all() and agent.adam_state()[2] == 2
    assert st2["approx_kl"] >= 0.0


def test_update_cfg5_minibatch_2048_vs_torch():
    """cfg5's per-GPU minibatch: 256 envs x num_steps 2048 / 32 minibatches / 8 GPUs = 2 048 rows
    (carla_config.h:28,31,133-138). Hundreds of wgrad chunks per layer and conv1's reductions over
    2 048 x 8 836 output pixels, against the fp32 PyTorch reference at the per-tensor bars of
    _check_grad; stats rtol 1e-4, total norm rtol 1e-4, parameters after the clipped Adam step atol
    2e-6. The reference takes ~12 s and ~11 GB of host memory on 8 threads."""
    torch.set_num_threads(16)
    L = CI.layout()
    p = CI.params(L)
    n = 2048
    rng = np.random.default_rng(11)
    bev = rng.integers(0, 256, size=(n, 15, 192, 192), dtype=np.uint8)
    f = lambda *shape: rng.uniform(-1, 1, shape).astype(np.float32)  # noqa: E731
    batch = (bev, f(n, 8), f(n, 3), f(n, 2) * 0.95, f(n) * 0.2, rng.standard_normal(n).astype(np.float32),
             rng.standard_normal(n).astype(np.float32), f(n) * 0.1)
    ag = ppo_amd.CarlaAgent(max_batch=n, seed=7)
    try:
        ag.load_params(p)
        ag.load_adam(np.zeros(L.P, np.float32), np.zeros(L.P, np.float32), 0)
        st, grad, newp = _run_update(ag, *batch)
    finally:
        ag.close()
    ref_g, ref_st, ref_total, ref_p, _, _ = TR.update(L, p, *batch, **CFG)
    stats = np.array([st[k] for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac")])
    np.testing.assert_allclose(stats[:5], ref_st[:5], rtol=1e-4, atol=2e-6)
    assert abs(stats[5] - ref_st[5]) <= 1.5 / n  # clipfrac: at most one row on the other side of the clip
    np.testing.assert_allclose(st["grad_norm"], ref_total, rtol=1e-4)
    _check_grad(L, grad, ref_g)
    np.testing.assert_allclose(newp, ref_p, rtol=0, atol=2e-6)


def test_update_argument_errors(agent):
    x = DeviceArray.from_numpy(np.zeros((1, 2), np.float32))
    with pytest.raises(ppo_amd.PPOError, match="n >= 2"):
        agent.update(DeviceArray.from_numpy(np.zeros((1, 15, 192, 192), np.uint8), np.uint8), x, x, x, x, x, x, x)


def test_update_with_one_rank_communicator_is_bit_identical():
    """ppo_carla_comm_init with world = 1 runs the distributed sequence (split advantage statistics,
    RCCL all-reduces of the advantage mean, sum of squares, gradient and loss stats); on one rank it
    must reproduce the communicator-free update bit for bit. The 2-rank exchange itself is covered
    by tests/test_carla_dist_gloo.py."""
    L = CI.layout()
    p = CI.params(L)
    n = 8
    rng = np.random.default_rng(3)
    bev = rng.integers(0, 256, size=(n, 15, 192, 192), dtype=np.uint8)
    f = lambda *shape: rng.uniform(-1, 1, shape).astype(np.float32)  # noqa: E731
    batch = (bev, f(n, 8), f(n, 3), f(n, 2) * 0.9, f(n) * 0.2, rng.standard_normal(n).astype(np.float32),
             rng.standard_normal(n).astype(np.float32), f(n) * 0.1)
    out = []
    for with_comm in (False, True):
        ag = ppo_amd.CarlaAgent(max_batch=n, seed=7)
        try:
            ag.load_params(p)
            if with_comm:
                ag.comm_init(ppo_amd.Agent.comm_unique_id(), 0, 1)
                ag.comm_broadcast_params(0)
            res = [_run_update(ag, *batch) for _ in range(2)]
            out.append(res)
        finally:
            ag.close()
    for (st0, g0, p0), (st1, g1, p1) in zip(*out):
        np.testing.assert_array_equal(g0, g1)
        np.testing.assert_array_equal(p0, p1)
        assert st0 == st1


def test_generic_wgrad_sample_groups_match_one_pass():
    """The generic fp32 weight-gradient kernel addresses its input with 32-bit buffer offsets, so an
    input of >= 0x70000000 bytes (conv2's 8 x 94 x 94 floats per sample: ~6.6 K rows) runs as sample
    groups whose sums are added in group order. wgrad_group_bytes lowers that limit so the group
    arithmetic runs at n = 24 (1.5 MB: conv2 in 5 groups of <= 5 samples, conv3 in 3 of <= 11, both
    with a ragged last group; the smaller layers in one pass): gradients within rel-L2 1e-5 per tensor of the one-pass generic kernel
    (another summation order of the same fp32 products), stepped parameters atol 1e-6."""
    L = CI.layout()
    p = CI.params(L)
    n = 24
    rng = np.random.default_rng(29)
    bev = rng.integers(0, 256, size=(n, 15, 192, 192), dtype=np.uint8)
    f = lambda *shape: rng.uniform(-1, 1, shape).astype(np.float32)  # noqa: E731
    batch = (bev, f(n, 8), f(n, 3), f(n, 2) * 0.95, f(n) * 0.2, rng.standard_normal(n).astype(np.float32),
             rng.standard_normal(n).astype(np.float32), f(n) * 0.1)
    out = {}
    for o in ("conv_wgrad=generic", "conv_wgrad=generic,wgrad_group_bytes=1500000"):
        ag = ppo_amd.CarlaAgent(max_batch=n, seed=7, options=o)
        try:
            ag.load_params(p)
            ag.load_adam(np.zeros(L.P, np.float32), np.zeros(L.P, np.float32), 0)
            out[o] = _run_update(ag, *batch)
        finally:
            ag.close()
    (s0, g0, p0), (s1, g1, p1) = out.values()
    for t in range(L.ntensors):
        o_, n_ = L.t_off[t], L.t_len[t]
        a, b = g1[o_:o_ + n_].astype(np.float64), g0[o_:o_ + n_].astype(np.float64)
        assert np.linalg.norm(a - b) <= 1e-5 * max(np.linalg.norm(b), 1e-30), t
    np.testing.assert_allclose(p1, p0, rtol=0, atol=1e-6)
    assert s0["pg_loss"] == s1["pg_loss"]  # the forward and the loss do not depend on the option


@pytest.mark.parametrize("opt", ["conv1_mfma=bx3"])
def test_conv1_split_bf16_update_vs_torch(opt):
    """conv1 (raw-byte input) with its products as split-bf16 MFMAs (conv1_mfma=bx3: the byte operand
    is exact in bf16, the fp32 operand's three pieces make every product exact; fp32 accumulation),
    n = 64 rows, against the fp32 PyTorch reference at the bars every CaRL update test uses
    (_check_grad per tensor, stats rtol 1e-4 with clipfrac within one row, total norm rtol 1e-4,
    stepped parameters atol 2e-6); the fp32-MFMA form (conv1_mfma=f32) runs the same batch and both
    errors are printed."""
    torch.set_num_threads(16)
    L = CI.layout()
    p = CI.params(L)
    n = 64
    rng = np.random.default_rng(23)
    bev = rng.integers(0, 256, size=(n, 15, 192, 192), dtype=np.uint8)
    f = lambda *shape: rng.uniform(-1, 1, shape).astype(np.float32)  # noqa: E731
    batch = (bev, f(n, 8), f(n, 3), f(n, 2) * 0.95, f(n) * 0.2, rng.standard_normal(n).astype(np.float32),
             rng.standard_normal(n).astype(np.float32), f(n) * 0.1)
    out = {}
    for o in ("conv1_mfma=f32", opt):
        ag = ppo_amd.CarlaAgent(max_batch=n, seed=7, options=o)
        try:
            ag.load_params(p)
            ag.load_adam(np.zeros(L.P, np.float32), np.zeros(L.P, np.float32), 0)
            out[o] = _run_update(ag, *batch)
        finally:
            ag.close()
    ref_g, ref_st, ref_total, ref_p, _, _ = TR.update(L, p, *batch, **CFG)
    (s0, g0, _), (s1, g1, p1) = out["conv1_mfma=f32"], out[opt]
    rel = lambda a, b: np.linalg.norm(a.astype(np.float64) - b) / max(np.linalg.norm(b.astype(np.float64)), 1e-30)  # noqa: E731
    print(f"\ngradient rel-L2 vs torch f32: conv1_mfma=f32 {rel(g0, ref_g):.2e}, {opt} {rel(g1, ref_g):.2e}")
    _check_grad(L, g1, ref_g)
    stats = np.array([s1[k] for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl", "approx_kl", "clipfrac")])
    np.testing.assert_allclose(stats[:5], ref_st[:5], rtol=1e-4, atol=2e-6)
    assert abs(stats[5] - ref_st[5]) <= 1.5 / n
    np.testing.assert_allclose(s1["grad_norm"], ref_total, rtol=1e-4)
    np.testing.assert_allclose(p1, ref_p, rtol=0, atol=2e-6)
