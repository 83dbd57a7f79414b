"""The persistent device-env rollout (k_rollout + k_values, csrc/ppo_rollout.hip) against the
per-step path (k_act3 + k_synth_step launches per step) through the C-ABI (ppo_set_rollout_mode).

The persistent kernel keeps the actor's weights in registers and runs obs -> actor -> Beta sample
-> env step for all T steps in one launch; the critic runs afterwards over the stored observations.
Both use the same arithmetic in the same order, so the whole rollout storage (obs, actions,
log-probs, rewards, dones, values), the env state, the episode statistics and -- after the shared
update -- the parameters must be bitwise equal. Covers ragged env blocks (E not a multiple of 16),
three observation widths (Hopper 11, HalfCheetah 17, Ant 105 with the Ant normalisation table) and
the 1000-step truncation with its next-step autoreset (9 x 128 steps)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")

BUFS = [("obs", "BUF_OBS", 1), ("actions", "BUF_ACTIONS", 2), ("logp", "BUF_LOGPROBS", 0),
        ("rewards", "BUF_REWARDS", 0), ("dones", "BUF_DONES", 0), ("values", "BUF_VALUES", 0)]


def snapshot(tr):
    E, T, O, A = tr.hcfg.num_envs, tr.hcfg.num_steps, tr.hcfg.obs_dim, tr.hcfg.act_dim
    out = {}
    for name, b, kind in BUFS:
        shape = (T, E, O) if kind == 1 else (T, E, A) if kind == 2 else (T, E)
        out[name] = tr.agent.buffer(getattr(ppo_amd, b), shape).numpy()
    out["next_obs"] = tr.next_obs.numpy()
    out["next_done"] = tr.next_done.numpy()
    return out


@pytest.mark.parametrize("agent,env_id,E,iters", [("ac", "HalfCheetah-v5", 200, 9), ("ac", "Hopper-v5", 37, 9),
                                                  ("ac", "HalfCheetah-v5", 998, 2), ("ac", "Ant-v5", 96, 3),
                                                  ("ppo", "HalfCheetah-v5", 37, 9),
                                                  ("ppo", "Hopper-v5", 20, 2), ("ppo", "Humanoid-v4", 40, 2)])
def test_persistent_rollout_bitwise_equals_per_step(agent, env_id, E, iters):
    """AC agent: the persistent rollout (k_rollout_v, the VALU form with 2 envs per workgroup, at
    E <= 512 and O <= 32 — E = 200 / 37 here; k_rollout, 16 envs per workgroup on MFMA, at E = 998
    and for Ant's O = 105) + k_values vs k_act3 + k_synth_step. PPO agent: k_rollout4 + k_values4 vs
    k_act4 (act_kernel=4) + k_synth_step(_wide), with the PPO wrapper chain (ppo:41-49) fused into
    both (Humanoid: O = 376, A = 17, two head tiles, actions clipped to [-0.4, 0.4])."""
    T = 128
    C = ppo_amd.ACPPOConfig if agent == "ac" else ppo_amd.PPOConfig
    cfg = C(env_id=env_id, num_envs=E, num_steps=T, num_minibatches=4, update_epochs=2, total_timesteps=E * T * iters)
    trs = [ppo_amd.Trainer(cfg, options="act_kernel=4"), ppo_amd.Trainer(cfg, options="act_kernel=4,rollout=per_step")]
    n_done = 0.0
    for it in range(iters):
        snaps, stats = [], []
        for tr in trs:
            tr.rollout()
            tr.agent.sync()
            snaps.append(snapshot(tr))
            stats.append(tr.env.episode_stats())
            tr.agent.compute_gae(tr.next_obs, tr.next_done)
            tr.agent.update(tr.lr_now(), want_stats=False)
            tr.iteration += 1
        for k in snaps[0]:
            np.testing.assert_array_equal(snaps[0][k], snaps[1][k], err_msg=f"iteration {it}: {k}")
        assert stats[0] == stats[1], it
        np.testing.assert_array_equal(trs[0].agent.params(), trs[1].agent.params(), err_msg=f"iteration {it}")
        n_done += snaps[0]["dones"].sum()
    if iters * T >= 1000:
        assert n_done == E  # the 1000-step truncation (and its autoreset) happened inside a rollout
    if agent == "ppo":
        for k, v in trs[0].wrappers.state().items():
            np.testing.assert_array_equal(v, trs[1].wrappers.state()[k], err_msg=k)
    for tr in trs:
        tr.close()


@pytest.mark.parametrize("env_id,E", [("HalfCheetah-v5", 512), ("HalfCheetah-v5", 1024), ("HalfCheetah-v5", 333),
                                      ("Hopper-v5", 64)])
def test_valu_rollout_bitwise_equals_mfma_rollout(env_id, E):
    """The N = 8 / N = 4 shards of the metric config (AC HalfCheetah, E = 512 / 1 024), an odd E (the
    last workgroup's second env absent) and Hopper (O = 11: one 16-wide input block, observation
    normalisation tables): the VALU rollout (rollout_kernel=valu: 2 envs per workgroup, v_fma_f32 /
    row_newbcast chains in the MFMA's k order, k_act3's LayerNorm / head partial-sum trees) against
    the MFMA rollout (rollout_kernel=mfma): every stored buffer, the env state and, after the shared
    update, the parameters bitwise equal over two iterations."""
    cfg = ppo_amd.ACPPOConfig(env_id=env_id, num_envs=E, num_steps=128, num_minibatches=1 if E % 4 else 4,
                              update_epochs=1, total_timesteps=E * 128 * 2)
    trs = [ppo_amd.Trainer(cfg, options="rollout_kernel=valu"), ppo_amd.Trainer(cfg, options="rollout_kernel=mfma")]
    for it in range(2):
        snaps = []
        for tr in trs:
            tr.rollout()
            tr.agent.sync()
            snaps.append(snapshot(tr))
            tr.agent.compute_gae(tr.next_obs, tr.next_done)
            tr.agent.update(tr.lr_now(), want_stats=False)
            tr.iteration += 1
        for k in snaps[0]:
            np.testing.assert_array_equal(snaps[0][k], snaps[1][k], err_msg=f"iteration {it}: {k}")
        assert trs[0].env.episode_stats() == trs[1].env.episode_stats()
        np.testing.assert_array_equal(trs[0].agent.params(), trs[1].agent.params())
    for tr in trs:
        tr.close()


def test_valu_rollout_bitwise_across_episode_ends():
    """The VALU rollout against the MFMA rollout over 1 152 steps per env (9 iterations of 128; the
    synthetic env truncates at 1 000 steps), so every env's autoreset branch (Philox reset of the
    state, episode bookkeeping) runs inside k_rollout_v: stored buffers, env state, episode
    statistics and parameters bitwise equal after every iteration."""
    E, T = 64, 128
    cfg = ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=E, num_steps=T, num_minibatches=2,
                              update_epochs=1, total_timesteps=E * T * 9)
    trs = [ppo_amd.Trainer(cfg, options="rollout_kernel=valu"), ppo_amd.Trainer(cfg, options="rollout_kernel=mfma")]
    finished = 0.0
    for it in range(9):
        snaps = []
        for tr in trs:
            tr.rollout()
            tr.agent.sync()
            snaps.append(snapshot(tr))
            tr.agent.compute_gae(tr.next_obs, tr.next_done)
            tr.agent.update(tr.lr_now(), want_stats=False)
            tr.iteration += 1
        for k in snaps[0]:
            np.testing.assert_array_equal(snaps[0][k], snaps[1][k], err_msg=f"iteration {it}: {k}")
        st = [tr.env.episode_stats() for tr in trs]  # (return sum, length sum, count); read-out resets them
        assert st[0] == st[1]
        finished += st[0][2]
        np.testing.assert_array_equal(trs[0].agent.params(), trs[1].agent.params())
    assert finished == E  # every env finished one episode (and was reset) inside the rollout
    for tr in trs:
        tr.close()


def test_persistent_rollout_metric_shape_properties():
    """The metric configuration (E=4096, T=128): the persistent path fills the storage with finite
    values, actions inside the action space, log-probs of the Beta policy, and is deterministic."""
    cfg = ppo_amd.ACPPOConfig(env_id="HalfCheetah-v5", num_envs=4096, total_timesteps=4096 * 128 * 4)
    res = []
    for _ in range(2):
        tr = ppo_amd.Trainer(cfg)
        tr.rollout()
        tr.agent.sync()
        res.append(snapshot(tr))
        tr.close()
    for k in res[0]:
        np.testing.assert_array_equal(res[0][k], res[1][k], err_msg=k)
    s = res[0]
    assert np.isfinite(s["values"]).all() and np.isfinite(s["logp"]).all()
    assert np.abs(s["actions"]).max() <= 1.0


@pytest.mark.parametrize("agent,env_id,E,T,mb", [("ac", "HalfCheetah-v5", 256, 128, 4), ("ppo", "Humanoid-v4", 64, 64, 32),
                                                 ("ppo", "HalfCheetah-v5", 1, 256, 4)])
def test_gradstep_fused_equals_split(agent, env_id, E, T, mb):
    """clip_grad_norm_ + Adam as one cooperative launch (k_gradstep, gradstep=fused: the norm slices,
    a grid barrier, the Adam blocks) against the two launches k_gradnorm + k_adam (gradstep=split,
    gradnorm=slices): the same functions in the same order, so parameters, Adam moments and the
    per-minibatch total norm are bitwise equal after two iterations (many minibatches: the barrier
    counter runs across launches)."""
    C = ppo_amd.ACPPOConfig if agent == "ac" else ppo_amd.PPOConfig
    cfg = C(env_id=env_id, num_envs=E, num_steps=T, num_minibatches=mb, update_epochs=2, total_timesteps=E * T * 4)
    trs = [ppo_amd.Trainer(cfg, options="gradstep=fused"), ppo_amd.Trainer(cfg, options="gradstep=split,gradnorm=slices")]
    for _ in range(2):
        st = [tr.iterate(want_stats=True) for tr in trs]
    np.testing.assert_array_equal(trs[0].agent.params(), trs[1].agent.params())
    m0, v0, s0 = trs[0].agent.adam_state()
    m1, v1, s1 = trs[1].agent.adam_state()
    np.testing.assert_array_equal(m0, m1)
    np.testing.assert_array_equal(v0, v1)
    assert s0 == s1
    assert st[0]["grad_norm"] == st[1]["grad_norm"]
    for tr in trs:
        tr.close()


@pytest.mark.parametrize("agent,env_id,E,T,mb", [("ac", "HalfCheetah-v5", 256, 128, 4), ("ppo", "Humanoid-v4", 64, 64, 32),
                                                 ("ppo", "HalfCheetah-v5", 1, 256, 4), ("ac", "Ant-v5", 96, 64, 2)])
def test_gradnorm_fold_matches_slices(agent, env_id, E, T, mb):
    """clip_grad_norm_'s sums of squares folded into k_colsum (gradnorm=fold: per-tile
    sums, the last tile of each tensor adds them in tile order through the agent-scope counter
    hand-off) against k_gradnorm's 16 slices per tensor (gradnorm=slices): the same values summed in
    another order, so the per-minibatch total norms agree to fp32 rounding and the parameters after
    two iterations stay within the update tests' bars; the fold is deterministic (two runs bitwise)."""
    C = ppo_amd.ACPPOConfig if agent == "ac" else ppo_amd.PPOConfig
    cfg = C(env_id=env_id, num_envs=E, num_steps=T, num_minibatches=mb, update_epochs=2, total_timesteps=E * T * 4)
    trs = [ppo_amd.Trainer(cfg, options="gradnorm=fold"), ppo_amd.Trainer(cfg, options="gradnorm=fold"),
           ppo_amd.Trainer(cfg, options="gradnorm=slices")]
    try:
        assert trs[0].agent.kernel_info().endswith("norm=k_colsum")
        assert trs[2].agent.kernel_info().endswith("norm=k_gradnorm")
        norms = [[], [], []]
        for _ in range(2):
            for i, tr in enumerate(trs):
                norms[i].append(tr.iterate(want_stats=True)["grad_norm"])
        p = [tr.agent.params() for tr in trs]
        np.testing.assert_array_equal(p[0], p[1])
        assert norms[0] == norms[1]
        np.testing.assert_allclose(norms[0], norms[2], rtol=1e-5)
        d = np.abs(p[0].astype(np.float64) - p[2])
        lr = float(cfg.learning_rate)
        assert (d > 2e-5).mean() < 1e-3 and d.max() < 2 * lr, ((d > 2e-5).sum(), d.max())
    finally:
        for tr in trs:
            tr.close()


@pytest.mark.parametrize("agent,env_id,E,T,mb,it", [("ac", "HalfCheetah-v5", 256, 128, 4, 3), ("ppo", "Humanoid-v4", 64, 64, 32, 3),
                                                    ("ppo", "HalfCheetah-v5", 1, 256, 4, 4), ("ac", "Ant-v5", 96, 64, 2, 3)])
def test_update_graph_equals_eager(agent, env_id, E, T, mb, it):
    """ppo_update's minibatch loop replayed as one captured hipGraph (update_graph=1: eager on the
    first call, captured on the second, replayed after) against the eager launches: the Adam step
    constants come from a device table written before each replay, everything else is the same
    launch sequence, so parameters, Adam moments and the per-minibatch stats are bitwise equal over
    several iterations with the annealed learning rate."""
    C = ppo_amd.ACPPOConfig if agent == "ac" else ppo_amd.PPOConfig
    cfg = C(env_id=env_id, num_envs=E, num_steps=T, num_minibatches=mb, update_epochs=2, total_timesteps=E * T * it)
    trs = [ppo_amd.Trainer(cfg, options="gradstep=split,update_graph=0"), ppo_amd.Trainer(cfg, options="gradstep=split,update_graph=1")]
    for i in range(it):
        st = [tr.iterate(want_stats=True) for tr in trs]
        np.testing.assert_array_equal(trs[0].agent.params(), trs[1].agent.params(), err_msg=f"iteration {i}")
        assert st[0] == st[1], i
    m0, v0, s0 = trs[0].agent.adam_state()
    m1, v1, s1 = trs[1].agent.adam_state()
    np.testing.assert_array_equal(m0, m1)
    np.testing.assert_array_equal(v0, v1)
    assert s0 == s1
    for tr in trs:
        tr.close()


@pytest.mark.parametrize("agent,env_id,E,T,mb", [("ac", "HalfCheetah-v5", 256, 128, 4), ("ppo", "HalfCheetah-v5", 1, 256, 4)])
def test_update_graph_back_to_back_and_snapshots(agent, env_id, E, T, mb):
    """update_graph=1 without a host sync between replays (want_stats=False: the Adam step table is
    restaged every replay while earlier copies may still be pending), and the checkpoint snapshot the
    CLI takes every iteration (ppo_snapshot_state on the context stream, ppo_read_snapshot from a
    writer thread while the next update is captured / replayed: ac:904-927). Parameters and Adam
    state are bitwise the eager run's, and every snapshot holds exactly the state after its iteration."""
    import ctypes
    import threading
    C = ppo_amd.ACPPOConfig if agent == "ac" else ppo_amd.PPOConfig
    it = 5
    cfg = C(env_id=env_id, num_envs=E, num_steps=T, num_minibatches=mb, update_epochs=2, total_timesteps=E * T * it)
    eager = ppo_amd.Trainer(cfg, options="update_graph=0")
    graph = ppo_amd.Trainer(cfg, options="update_graph=1")
    lib = ppo_amd.lib()
    P = graph.agent.num_params
    ref, snaps, errs = [], [], []
    for i in range(it):
        eager.iterate(want_stats=False)
        ref.append(eager.agent.params())
    graph.iterate(want_stats=False)
    for k in range(it):
        ppo_amd.check(lib.ppo_snapshot_state(graph.agent.h))
        p = np.zeros(P, np.float32)

        def reader(p=p):
            st = ctypes.c_long()
            if lib.ppo_read_snapshot(graph.agent.h, p.ctypes.data, None, None,
                                     P, ctypes.byref(st)) != 0:
                errs.append(lib.ppo_last_error().decode())
        th = threading.Thread(target=reader)
        th.start()
        if k + 1 < it:  # the next iteration (its update captured on the second call) beside the reader
            graph.iterate(want_stats=False)
        th.join()
        snaps.append(p)
    assert not errs, errs
    for k in range(it):
        np.testing.assert_array_equal(snaps[k], ref[k], err_msg=f"snapshot after iteration {k}")
    graph.agent.sync()
    np.testing.assert_array_equal(graph.agent.params(), eager.agent.params())
    m0, v0, s0 = eager.agent.adam_state()
    m1, v1, s1 = graph.agent.adam_state()
    np.testing.assert_array_equal(m0, m1)
    np.testing.assert_array_equal(v0, v1)
    assert s0 == s1
    for tr in (eager, graph):
        tr.close()
