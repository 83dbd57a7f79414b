"""GPU parity of the CaRL CNN agent's forward through the C-ABI (ppo_carla_forward)
against the LibTorch replay of include/carla/carla_model.h (golden case carla_act) and the C oracle.

Tolerances: convolutions and Linear layers are fp32 MFMA chains in a different summation order from
LibTorch's (1.2 M parameters, K up to 1 280) — alpha / beta / value rtol 1e-4, log-prob and entropy
atol 2e-4; sampled actions vs the oracle (same Philox draws, alpha / beta differ in the last bits)
atol 2e-4. Batch composition: bitwise (every output pixel runs the same MFMA chain for any n)."""
import numpy as np
import pytest

import carla_inputs as CI
from golden_io import load_case

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402


def run(agent, bev, meas, vmeas, act=None, mode="sample", env_base=0, step_id=0):
    d = [DeviceArray.from_numpy(bev, np.uint8), DeviceArray.from_numpy(meas), DeviceArray.from_numpy(vmeas)]
    a = DeviceArray.from_numpy(act) if act is not None else None
    out = agent.forward(*d, actions=a, sample_type=mode, env_base=env_base, step_id=step_id)
    return [o.numpy() for o in out]


@pytest.fixture(scope="module")
def carla():
    ppo_amd.set_device(0)
    meta, gold = load_case("carla_act")
    L = CI.layout()
    p = CI.params(L)
    ag = ppo_amd.CarlaAgent(max_batch=16, seed=7)
    assert ag.layout.P == L.P == meta["P"]
    ag.load_params(p)
    yield ag, L, p, meta, gold
    ag.close()


def test_forward_given_mean_roach_vs_golden(carla):
    ag, L, p, meta, g = carla
    bev, meas, vmeas, act = CI.inputs(meta["N"])
    a, lp, ent, v, al, be = run(ag, bev, meas, vmeas, act)
    np.testing.assert_allclose(al, g["alpha"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(be, g["beta"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(v, g["value"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(lp, g["logprob"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(ent, g["entropy"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(a, g["action_roundtrip"], rtol=1e-6, atol=1e-6)
    am, lpm = run(ag, bev, meas, vmeas, mode="mean")[:2]
    np.testing.assert_allclose(am, g["mean_action"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(lpm, g["mean_logprob"], rtol=1e-4, atol=2e-4)
    ar, lpr = run(ag, bev, meas, vmeas, mode="roach")[:2]
    np.testing.assert_allclose(ar, g["roach_action"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(lpr, g["roach_logprob"], rtol=1e-4, atol=2e-4)


def test_sample_vs_oracle_and_batch_independence(carla):
    ag, L, p, meta, g = carla
    n = 8
    bev, meas, vmeas, _ = CI.inputs(n)
    a, lp, ent, v, al, be = run(ag, bev, meas, vmeas, mode="sample", env_base=5, step_id=11)
    o = CI.oracle_forward(L, p, bev, meas, vmeas, 0, seed=7, env_base=5, step_id=11)
    np.testing.assert_allclose(al, o["alpha"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(v, o["value"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(a, o["action"], rtol=1e-4, atol=2e-4)
    np.testing.assert_allclose(lp, o["logprob"], rtol=1e-4, atol=5e-4)
    assert np.all(np.abs(a) <= 1.0)
    # rows 2..4 alone, env_base shifted to match: bitwise the same draws and values
    a2, lp2, ent2, v2, al2, be2 = run(ag, bev[2:5], meas[2:5], vmeas[2:5], mode="sample", env_base=7, step_id=11)
    np.testing.assert_array_equal(a2, a[2:5])
    np.testing.assert_array_equal(v2, v[2:5])
    np.testing.assert_array_equal(lp2, lp[2:5])


def test_errors(carla):
    ag = carla[0]
    bev, meas, vmeas, _ = CI.inputs(1)
    big = np.repeat(bev, 17, axis=0)
    with pytest.raises(ppo_amd.PPOError, match="max_batch"):
        run(ag, big, np.repeat(meas, 17, 0), np.repeat(vmeas, 17, 0), mode="mean")
    with pytest.raises(ppo_amd.PPOError):
        ppo_amd.CarlaAgent(max_batch=4, bev=128)  # roach encoder needs 256 x 2 x 2 at the end


def test_staged_conv1_kernels_match_generic():
    """conv1 runs through k_conv_img2 / k_wgrad_img2 (uint8 patch staged in LDS, ds_read_u8 gathers,
    two output columns per MFMA column for OC = 8) and conv2's input gradient through k_dgrad_s2 (dZ
    region staged in LDS); with the create option "conv1=generic" the generic k_conv / k_wgrad / k_dgrad
    gather from global memory. Forward: the real taps in k_conv's order, the extra taps with exact
    zero weights (the f32 MFMA accumulates as a sequential fma chain), so every output is bitwise
    equal (n = 7: partial tiles, 94 = 2 x 32 + 30 = 5 x 16 + 14). Update: k_dgrad_s2 keeps k_dgrad's chain (bitwise), so every gradient tensor
    but conv1's is bitwise equal; conv1's weight and bias gradients sum the 7 x 8 836 pixels in
    another order (relative L2 < 1e-5); the stepped parameters then differ through the clip
    coefficient (atol 1e-7)."""
    import carla_torch_ref  # noqa: F401  (skip like the update tests when torch is absent)
    n = 7
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(n)
    rng = np.random.default_rng(3)
    old_logp = rng.normal(-2.0, 0.3, n).astype(np.float32)
    adv = rng.normal(0.0, 1.0, n).astype(np.float32)
    ret = rng.normal(0.0, 1.0, n).astype(np.float32)
    old_v = rng.normal(0.0, 1.0, n).astype(np.float32)
    outs = []
    for opt in ("conv1=generic", "conv1=staged,conv_dgrad=staged,conv_wgrad=generic,conv_fwd=generic"):
        ag = ppo_amd.CarlaAgent(max_batch=16, seed=7, options=opt)
        ag.load_params(p)
        res = [run(ag, bev, meas, vmeas, mode=m, env_base=3, step_id=5) for m in ("sample", "mean", "roach")]
        res.append(run(ag, bev, meas, vmeas, act))
        d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                       for x in (meas, vmeas, act, old_logp, adv, ret, old_v)]
        ag.update(*d, lr=3e-4, clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5)
        res.append([ag.last_grad(), ag.params()])
        outs.append(res)
        ag.close()
    for r0, r1 in zip(outs[0][:4], outs[1][:4]):
        for x0, x1 in zip(r0, r1):
            np.testing.assert_array_equal(x0, x1)
    (g0, p0), (g1, p1) = outs[0][4], outs[1][4]
    conv1 = {L.conv_w[0], L.conv_b[0]}
    for t in range(L.ntensors):
        o, m = L.t_off[t], L.t_len[t]
        if o in conv1:
            r = np.linalg.norm((g1[o:o + m] - g0[o:o + m]).astype(np.float64)) / np.linalg.norm(g0[o:o + m])
            assert r < 1e-5, (t, r)
        else:
            np.testing.assert_array_equal(g1[o:o + m], g0[o:o + m])
    np.testing.assert_allclose(p1, p0, rtol=0, atol=1e-7)


@pytest.mark.parametrize("opts,layers", [(("conv_dgrad=staged", "conv_dgrad=quad"), (0, 1)),
                                         (("conv_wgrad=generic", "conv_wgrad=tiled"), (1, 2)),
                                         (("deep_dgrad=gather", "deep_dgrad=col"), (0, 1, 2, 3, 4))])
def test_conv2_backward_forms_match(opts, layers):
    """conv_dgrad=quad (conv2: k_dgrad_q, the four stride-2 parity classes as the columns of one GEMM
    over quads, k = (tap, oc) with the missing taps as zero weights; conv3: k_dgrad_q2, the classes as
    separate GEMMs sharing each dZ operand) against k_dgrad_s2 / k_dgrad (conv_dgrad=staged): conv3's
    and conv2's input gradients feed only conv2's and conv1's weight gradients (and conv2's input
    gradient), so every other gradient tensor is bitwise equal and those agree within fp32 summation
    noise (rel-L2 < 1e-5). conv_wgrad=tiled (k_wgrad_t for conv2, k_wgrad_t2 for conv3: dZ tile and
    input patch staged in LDS, one partial per persistent workgroup) against the generic k_wgrad: only
    conv2's and conv3's own weight and bias gradients differ, within the same bar. deep_dgrad=col (conv6's
    input gradient as a dense GEMM into columns + k_col2im) against k_dgrad: every conv layer's
    gradient below conv6 moves (conv6's own weight gradient and the MLP's stay bitwise). n = 7 covers the partial tiles (47 = 2 x 16 + 15 quads per
    edge; 45 = 5 x 8 + 5 and 2 x 16 + 13 output pixels) and a grid with fewer tiles than workgroups."""
    import carla_torch_ref  # noqa: F401
    n = 7
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(n)
    rng = np.random.default_rng(5)
    old_logp = rng.normal(-2.0, 0.3, n).astype(np.float32)
    adv = rng.normal(0.0, 1.0, n).astype(np.float32)
    ret = rng.normal(0.0, 1.0, n).astype(np.float32)
    old_v = rng.normal(0.0, 1.0, n).astype(np.float32)
    outs = []
    for opt in opts:
        ag = ppo_amd.CarlaAgent(max_batch=16, seed=7, options=opt)
        ag.load_params(p)
        d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                       for x in (meas, vmeas, act, old_logp, adv, ret, old_v)]
        ag.update(*d, lr=3e-4, clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5)
        outs.append((ag.last_grad(), ag.params()))
        ag.close()
    (g0, p0), (g1, p1) = outs
    moved = {o for i in layers for o in (L.conv_w[i], L.conv_b[i])}
    for t in range(L.ntensors):
        o, m = L.t_off[t], L.t_len[t]
        if o in moved:
            r = np.linalg.norm((g1[o:o + m] - g0[o:o + m]).astype(np.float64)) / np.linalg.norm(g0[o:o + m])
            assert r < 1e-5, (t, r)
        else:
            np.testing.assert_array_equal(g1[o:o + m], g0[o:o + m])
    np.testing.assert_allclose(p1, p0, rtol=0, atol=1e-7)


def test_tiled_conv2_forward_matches_generic():
    """conv_fwd=tiled (k_conv_t: input patch staged in LDS, weights in registers, k = (tap, ic)) against
    the generic k_conv: the same fp32 products in another k order, so the forward (mean mode: value,
    Beta concentrations, log-prob) agrees within fp32 summation noise, and after one update every
    gradient tensor within rel-L2 1e-4 and the stepped parameters within 1e-6 (n = 7: partial tiles,
    45 = 5 x 8 + 5 rows and 2 x 16 + 13 columns)."""
    import carla_torch_ref  # noqa: F401
    n = 7
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(n)
    rng = np.random.default_rng(6)
    old_logp = rng.normal(-2.0, 0.3, n).astype(np.float32)
    adv = rng.normal(0.0, 1.0, n).astype(np.float32)
    ret = rng.normal(0.0, 1.0, n).astype(np.float32)
    old_v = rng.normal(0.0, 1.0, n).astype(np.float32)
    outs = []
    for opt in ("conv_fwd=generic", "conv_fwd=tiled"):
        ag = ppo_amd.CarlaAgent(max_batch=16, seed=7, options=opt)
        ag.load_params(p)
        fwd = run(ag, bev, meas, vmeas, act)
        d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                       for x in (meas, vmeas, act, old_logp, adv, ret, old_v)]
        ag.update(*d, lr=3e-4, clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5)
        outs.append((fwd, ag.last_grad(), ag.params()))
        ag.close()
    (f0, g0, p0), (f1, g1, p1) = outs
    for x0, x1 in zip(f0, f1):
        np.testing.assert_allclose(x1, x0, rtol=1e-4, atol=1e-5)
    for t in range(L.ntensors):
        o, m = L.t_off[t], L.t_len[t]
        nrm = np.linalg.norm(g0[o:o + m].astype(np.float64))
        if nrm == 0:
            continue
        r = np.linalg.norm((g1[o:o + m] - g0[o:o + m]).astype(np.float64)) / nrm
        assert r < 1e-4, (t, r)
    np.testing.assert_allclose(p1, p0, rtol=0, atol=1e-6)


@pytest.mark.parametrize("opts", [("conv1=staged", "conv1=packed,conv1_mfma=f32"),
                                  ("conv1=packed,conv1_mfma=f32", "conv1=packed,conv1_mfma=bx3")])
def test_packed_conv1_matches_staged(opts):
    """conv1=packed (k_conv_img3: the taps of a 16-wide MFMA k block ordered so that each lane group's
    four k-steps are four consecutive patch bytes of one kernel row, one ds_read_b32 per B quadruple,
    A operands from a pre-arranged weight table) computes every product as k_conv_img2 does (u8 / 255
    times the same weight) in another k order: forward outputs within fp32 summation noise of the
    staged kernel (n = 7, partial tiles; every sampling mode), the update's gradients per tensor
    within rel-L2 1e-5, the stepped parameters within 1e-6. Golden / oracle / torch parity of the
    packed path itself: the module tests above run on the default conv1 form. The same bars hold
    between conv1's fp32-MFMA and split-bf16 forms (conv1_mfma=bx3: exact products of the byte operand
    and the weights' three bf16 pieces on 16x16x32 bf16 MFMAs, forward and weight gradient)."""
    import carla_torch_ref  # noqa: F401
    n = 7
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(n)
    rng = np.random.default_rng(4)
    old_logp = rng.normal(-2.0, 0.3, n).astype(np.float32)
    adv = rng.normal(0.0, 1.0, n).astype(np.float32)
    ret = rng.normal(0.0, 1.0, n).astype(np.float32)
    old_v = rng.normal(0.0, 1.0, n).astype(np.float32)
    outs = []
    for opt in opts:
        ag = ppo_amd.CarlaAgent(max_batch=16, seed=7, options=opt)
        ag.load_params(p)
        res = [run(ag, bev, meas, vmeas, mode=m, env_base=3, step_id=5) for m in ("sample", "mean", "roach")]
        res.append(run(ag, bev, meas, vmeas, act))
        d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                       for x in (meas, vmeas, act, old_logp, adv, ret, old_v)]
        ag.update(*d, lr=3e-4, clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5)
        res.append([ag.last_grad(), ag.params()])
        outs.append(res)
        ag.close()
    for r0, r1 in zip(outs[0][:4], outs[1][:4]):
        for x0, x1 in zip(r0, r1):
            np.testing.assert_allclose(x1, x0, rtol=2e-5, atol=2e-6)
    (g0, p0), (g1, p1) = outs[0][4], outs[1][4]
    for t in range(L.ntensors):
        o, m = L.t_off[t], L.t_len[t]
        nr = np.linalg.norm(g0[o:o + m])
        if nr > 0:
            r = np.linalg.norm((g1[o:o + m] - g0[o:o + m]).astype(np.float64)) / nr
            assert r < 1e-5, (t, r)
    # Adam's first step normalises g / |g|: a few near-zero gradient entries move by up to ~lr / 1000
    np.testing.assert_allclose(p1, p0, rtol=0, atol=1e-6)


def test_unaligned_image_pointer(carla):
    """The staged / packed first-layer kernels load the uint8 image as dwords: an image pointer that is
    not 4-byte aligned takes the generic gather path. It gives the staged kernel's outputs bitwise
    (conv1=staged keeps k_conv's MFMA chains), and the default (packed) outputs within fp32 noise."""
    ag, L, p = carla[0], carla[1], carla[2]
    n = 3
    bev, meas, vmeas, _ = CI.inputs(n)
    packed = run(ag, bev, meas, vmeas, mode="mean")
    ag_s = ppo_amd.CarlaAgent(max_batch=16, seed=7, options="conv1=staged")
    ag_s.load_params(p)
    ref = run(ag_s, bev, meas, vmeas, mode="mean")
    ag_s.close()
    for r, o in zip(ref, packed):
        np.testing.assert_allclose(o, r, rtol=2e-5, atol=2e-6)
    raw = np.zeros(bev.size + 4, np.uint8)
    raw[1:1 + bev.size] = bev.ravel()
    buf = DeviceArray.from_numpy(raw, np.uint8)
    shifted = DeviceArray.wrap(buf.ptr + 1, bev.shape, np.uint8)
    out = ag.forward(shifted, DeviceArray.from_numpy(meas), DeviceArray.from_numpy(vmeas), sample_type="mean")
    for r, o in zip(ref, out):
        np.testing.assert_array_equal(o.numpy(), r)


@pytest.mark.parametrize("n", [7, 16, 32])
def test_fused_tail_matches_layer_kernels(n):
    """Rollout-sized batches (n <= 64) run the MLP tail after the CNN — state MLP, linear, value and
    policy heads, the Beta head — as k_carla_tail: one cooperative launch with a grid barrier between
    dependency stages ("tail=fused", the default), or one launch per stage ("tail=staged"). Each
    Linear work item repeats k_conv's MFMA chains over the same 128-wide k chunks and adds the chunk
    partials in k_conv_fin's order, so every output (and the update's forward activations) equals the
    per-layer kernels' ("tail=layers") bit for bit, in every sampling mode."""
    L = CI.layout()
    p = CI.params(L)
    bev, meas, vmeas, act = CI.inputs(n)
    outs = {}
    for opt in ("tail=layers", "tail=fused", "tail=staged"):
        ag = ppo_amd.CarlaAgent(max_batch=64, seed=7, options=opt)
        ag.load_params(p)
        res = [run(ag, bev, meas, vmeas, mode=m, env_base=3, step_id=5) for m in ("sample", "mean", "roach")]
        res.append(run(ag, bev, meas, vmeas, act))
        if n <= 16:
            rng = np.random.default_rng(5)
            extra = [rng.normal(-2.0, 0.3, n), rng.normal(0.0, 1.0, n), rng.normal(0.0, 1.0, n), rng.normal(0.0, 1.0, n)]
            d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                           for x in [meas, vmeas, act] + extra]
            ag.update(*d, lr=3e-4, clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5)
            res.append([ag.last_grad(), ag.params()])
        outs[opt] = res
        ag.close()
    for opt in ("tail=fused", "tail=staged"):
        for r0, r1 in zip(outs["tail=layers"], outs[opt]):
            for x0, x1 in zip(r0, r1):
                np.testing.assert_array_equal(x1, x0)


def test_packed_conv1_odd_block_counts_match_generic():
    """conv1's packed table holds IC * K kernel rows in 16-tap blocks of two rows; its split-bf16 loop
    reads the blocks in pairs, so channel counts with an odd block count (IC = 5: 13 blocks, IC = 13:
    33) get a zero padding block. The packed bx3 forward and update at IC = 5, then IC = 13 in the same
    process (a later context needs more dynamic LDS than the first one: the kernel's LDS limit is set
    for the largest size the launch accepts), against the generic fp32 kernels on the same parameters:
    outputs rtol 2e-5 / atol 2e-6, gradients per tensor within rel-L2 1e-5."""
    n = 5
    rng = np.random.default_rng(41)
    for ch in (5, 13):
        bev = rng.integers(0, 256, size=(n, ch, 192, 192), dtype=np.uint8)
        meas = rng.uniform(-1, 1, (n, 8)).astype(np.float32)
        vmeas = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
        act = rng.uniform(-0.9, 0.9, (n, 2)).astype(np.float32)
        tail = [rng.normal(-2.0, 0.3, n), rng.normal(0, 1, n), rng.normal(0, 1, n), rng.normal(0, 1, n)]
        tail = [t.astype(np.float32) for t in tail]
        outs, p = [], None
        for opt in ("conv1=generic,conv1_mfma=f32", "conv1=packed,conv1_mfma=bx3"):
            ag = ppo_amd.CarlaAgent(max_batch=8, obs_channels=ch, seed=7, options=opt)
            try:
                if p is None:
                    p = ag.params()
                ag.load_params(p)
                res = [run(ag, bev, meas, vmeas, mode="mean"), run(ag, bev, meas, vmeas, act)]
                d = [DeviceArray.from_numpy(bev, np.uint8)] + [DeviceArray.from_numpy(np.ascontiguousarray(x, np.float32))
                                                               for x in (meas, vmeas, act, *tail)]
                ag.update(*d, lr=3e-4, clip_coef=0.2, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5)
                res.append(ag.last_grad())
                lay = ag.layout
                outs.append(res)
            finally:
                ag.close()
        for r0, r1 in zip(outs[0][:2], outs[1][:2]):
            for x0, x1 in zip(r0, r1):
                np.testing.assert_allclose(x1, x0, rtol=2e-5, atol=2e-6)
        g0, g1 = outs[0][2], outs[1][2]
        for t in range(lay.ntensors):
            o, m = lay.t_off[t], lay.t_len[t]
            nr = np.linalg.norm(g0[o:o + m].astype(np.float64))
            if nr > 0:
                assert np.linalg.norm((g1[o:o + m] - g0[o:o + m]).astype(np.float64)) / nr < 1e-5, (ch, t)
