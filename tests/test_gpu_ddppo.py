"""DD-PPO preemption on the device path (ac:570-583, :629, :680-693, :759-810) through the C-ABI:
a partial collection of Tc < num_steps steps per env.

  GAE: the reference's loop runs t = Tc-1 .. 0 and bootstraps t = Tc-1 from the STORED step Tc
    (values[Tc], dones[Tc]: t != num_steps - 1, ac:765-774) -- bit-exact against the oracle's GAE
    on the first Tc steps with that bootstrap.
  Update: each epoch's permutation covers the Tc * E collected samples and is repeated and
    truncated to the per-device batch (b_inds.repeat(ceil(B / Bc))[:B], ac:805-810).
    ppo_update_ex(Tc) must equal, bit for bit, ppo_update with those index lists built here from the
    oracle's Feistel permutation, and the oracle's update with the same lists within the
    full-iteration bar of test_full_iteration_vs_oracle (atol 2e-5).
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402
from test_gpu_parity import fill_storage, make_agent, random_params  # noqa: E402


def repeat_truncate(perm, B):
    """b_inds.repeat(num_repeat)[:B] with num_repeat = ceil(B / Bc) (ac:806-809)"""
    Bc = perm.size
    return np.tile(perm, (B + Bc - 1) // Bc)[:B]


@pytest.mark.parametrize("Tc", [1, 5, 11, 16])
def test_partial_collection_gae_bootstraps_from_the_stored_step(Tc):
    T, E = 16, 96
    rng = np.random.default_rng(7 + Tc)
    r = rng.standard_normal((T, E)).astype(np.float32)
    v = rng.standard_normal((T, E)).astype(np.float32)
    dn = (rng.random((T, E)) < 0.1).astype(np.float32)
    nv = rng.standard_normal(E).astype(np.float32)
    nd = (rng.random(E) < 0.5).astype(np.float32)
    ag = make_agent(1, 17, 6, 256, E, T=T, MB=2, EP=1)
    try:
        ag.buffer(ppo_amd.BUF_REWARDS, (T, E)).upload(r)
        ag.buffer(ppo_amd.BUF_VALUES, (T, E)).upload(v)
        ag.buffer(ppo_amd.BUF_DONES, (T, E)).upload(dn)
        ag.gae_from_values(DeviceArray.from_numpy(nv), DeviceArray.from_numpy(nd), nsteps=Tc)
        if Tc < T:
            oa, orr = O.gae(r[:Tc], v[:Tc], dn[:Tc], v[Tc], dn[Tc], 0.99, 0.95)
        else:  # a full collection: the bootstrap value and done after the last step
            oa, orr = O.gae(r, v, dn, nv, nd, 0.99, 0.95)
        np.testing.assert_array_equal(ag.buffer(ppo_amd.BUF_ADVANTAGES, (T, E)).numpy()[:Tc], oa)
        np.testing.assert_array_equal(ag.buffer(ppo_amd.BUF_RETURNS, (T, E)).numpy()[:Tc], orr)
    finally:
        ag.close()


@pytest.mark.parametrize("Tc", [3, 5, 13])
def test_partial_collection_update_repeats_and_truncates_the_permutation(Tc):
    T, E, MB, EP, it = 16, 64, 2, 2, 3
    O_, A, H = 17, 6, 256
    B = T * E
    rng = np.random.default_rng(30 + Tc)
    L = O.layout_init(1, O_, A, H)
    p = random_params(L, rng)
    obs = rng.standard_normal((B, O_)).astype(np.float32)
    act = rng.uniform(-0.95, 0.95, (B, A)).astype(np.float32)
    logp = (rng.standard_normal(B) * 0.3 - 4.0).astype(np.float32)
    adv = rng.standard_normal(B).astype(np.float32)
    ret = rng.standard_normal(B).astype(np.float32)
    val = rng.standard_normal(B).astype(np.float32) * 0.1
    perms = np.stack([repeat_truncate(O.perm(Tc * E, 1, 0, it * EP + e), B) for e in range(EP)]).astype(np.int32)
    assert perms.max() < Tc * E and perms.shape == (EP, B)
    res = []
    for explicit in (False, True):
        ag = make_agent(1, O_, A, H, E, T=T, MB=MB, EP=EP, clip=0.1)
        try:
            ag.load_params(p)
            fill_storage(ag, T, E, obs, act, logp, adv, ret, val)
            ag.set_iteration(it)
            if explicit:
                st = ag.update(2.5e-4, perms=DeviceArray.from_numpy(perms.reshape(-1), np.int32))
            else:
                st = ag.update(2.5e-4, num_steps_collected=Tc)
            res.append((ag.params(), ag.last_grad(), st))
        finally:
            ag.close()
    (p0, g0, s0), (p1, g1, s1) = res
    np.testing.assert_array_equal(g0, g1)
    np.testing.assert_array_equal(p0, p1)
    assert s0 == s1
    lcfg = O.LossCfg(0.1, 0.01, 0.5, 1, 1)
    op, _, _, _, _ = O.update(L, p, np.zeros(L.P), np.zeros(L.P), 0, obs, act, logp, adv, ret, val, EP, MB, 2.5e-4,
                              0.5, 1e-5, lcfg, seed=1, rank=0, epoch_counter0=it * EP, perms=perms.astype(np.int64))
    np.testing.assert_allclose(p0, op, rtol=0, atol=2e-5)


def test_partial_collection_step_count_is_checked():
    ag = make_agent(1, 17, 6, 256, 8, T=4, MB=1, EP=1)
    try:
        with pytest.raises(ppo_amd.PPOError, match="collected step count"):
            ag.update(1e-4, num_steps_collected=5)
    finally:
        ag.close()
