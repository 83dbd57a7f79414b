"""GPU parity at the widths the reference builds, straight against the LibTorch-replay golden vectors
(oracle/ref_harness.cpp width_cases()), through the C-ABI:

  ac256   AC agent, 2x256 LayerNorm trunks + Beta heads (ac:150-249), HalfCheetah O=17 / A=6
          -> k_act (API act), k_act3 (rollout act), k_upd<256, LN_BETA> + k_dwf (update)
  ant256  the same agent at Ant-v5 O=105 / A=8 (cfg4)
  hum376  PPO agent, 2x64 tanh + Normal (ppo:120-157), Humanoid-v4 O=376 / A=17 (cfg2)
          -> k_act (API act), k_act4 (rollout act: K-split, wide input), k_upd2 + k_dw2 (update)
  gae_long / gae_t{1,7,33}  k_gae at cfg2's T=2048 (E=1024) and at ragged T (32-step load chunks)

Tolerances (fp32; MFMA f32 chains vs LibTorch's CPU GEMMs, the same bars as test_gpu_parity.py):
  log-probs / entropies / values     rtol 2e-5 .. 1e-4
  raw gradient                        relative L2 < 2e-4 overall, < 2e-3 per tensor
  parameters after 1 / 3 Adam steps   atol 2e-6 / 6e-6
  GAE                                 bit-exact
"""
import numpy as np
import pytest

import oracle_lib as O

from golden_inputs import column_fnv, gae_long_inputs, hash_params
from golden_io import load_case

pytestmark = pytest.mark.gpu

ppo_amd = pytest.importorskip("ppo_amd")
from ppo_amd import DeviceArray  # noqa: E402

WIDTH_CASES = [("ac256", 1), ("ant256", 1), ("hum376", 0)]


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)


def agent_for(meta, E, T=1, MB=1, EP=1, **kw):
    hc = ppo_amd.HipConfig(meta["kind"], meta["O"], meta["A"], meta["H"], E, T, MB, EP, 0.99, 0.95,
                           kw.get("clip", 0.2), kw.get("ent", 0.01), kw.get("vf", 0.5), kw.get("mgn", 0.5),
                           kw.get("eps", 1e-5), 1, 1, 1, 0, 1)
    return ppo_amd.Agent(hc, options=kw.get("options"))


def golden_params(pre):
    meta, _ = load_case(pre + "_act")
    L = ppo_amd.agent_layout(meta["kind"], meta["O"], meta["A"], meta["H"])
    return meta, hash_params(L, meta["hash_base"], meta.get("hi", 1.0), meta.get("lo", -1.0))


@pytest.mark.parametrize("pre,kind", WIDTH_CASES)
def test_act_vs_golden_at_reference_width(pre, kind):
    meta, p = golden_params(pre)
    _, d = load_case(pre + "_act")
    n = d["x"].shape[0]
    ag = agent_for(meta, n)
    ag.load_params(p)
    np.testing.assert_array_equal(ag.params(), p)
    x, a = DeviceArray.from_numpy(d["x"]), DeviceArray.from_numpy(d["action"])
    act, lp, ent, v = ag.get_action_and_value(x, ppo_amd.PPO_GIVEN, a)
    np.testing.assert_allclose(lp.numpy(), d["logprob"], rtol=2e-5, atol=1e-4)
    np.testing.assert_allclose(ent.numpy(), d["entropy"], rtol=2e-5, atol=1e-4)
    np.testing.assert_allclose(v.numpy(), d["value"], rtol=2e-5, atol=2e-5)
    am, lpm, _, _ = ag.get_action_and_value(x, ppo_amd.PPO_MEAN)
    if kind == 1:
        np.testing.assert_allclose(act.numpy(), d["action_roundtrip"], rtol=0, atol=2e-7)
        np.testing.assert_allclose(am.numpy(), d["mean_action"], rtol=1e-5, atol=2e-6)
        np.testing.assert_allclose(lpm.numpy(), d["mean_logprob"], rtol=2e-5, atol=1e-4)
    else:
        np.testing.assert_allclose(am.numpy(), d["mean"], rtol=1e-5, atol=2e-6)
    ag.close()
    # the rollout act kernel (the one the trainer launches every step) on the same rows, as rollout
    # step 0 of a context with E = n envs: the stored value vs the golden critic output, the sampled
    # actions and their log-probs vs the oracle drawing the same Philox counters
    ag = agent_for(meta, n, T=2)
    ag.load_params(p)
    done = DeviceArray.from_numpy(np.zeros(n, np.float32))
    ag.rollout_act(0, 0, n, x, done)
    ag.rollout_values()  # the critic pass (deferred where values_mfma=bx6 applies)
    np.testing.assert_array_equal(ag.buffer(ppo_amd.BUF_OBS, (2, n, meta["O"])).numpy()[0], d["x"])
    np.testing.assert_allclose(ag.buffer(ppo_amd.BUF_VALUES, (2, n)).numpy()[0], d["value"], rtol=2e-5, atol=2e-5)
    L = O.layout_init(meta["kind"], meta["O"], meta["A"], meta["H"])
    oa, olp, _, _ = O.get_action_and_value(L, p, d["x"], 0, seed=1, rank=0, env_base=0, step_id=0)
    np.testing.assert_allclose(ag.buffer(ppo_amd.BUF_ACTIONS, (2, n, meta["A"])).numpy()[0], oa, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(ag.buffer(ppo_amd.BUF_LOGPROBS, (2, n)).numpy()[0], olp, rtol=1e-4, atol=1e-3)
    ag.close()


@pytest.mark.parametrize("pre,kind,opts", [c + (None,) for c in WIDTH_CASES] +
                         [("ac256", 1, "upd_mfma=32"), ("ant256", 1, "upd_mfma=32")])
def test_update_vs_golden_at_reference_width(pre, kind, opts):
    """The update at the reference widths against the LibTorch golden; the AC agent also through
    k_upd32 (create option upd_mfma=32)."""
    meta, p = golden_params(pre)
    mu, d = load_case(pre + "_update")
    M = mu["M"]
    ag = agent_for(meta, M, clip=mu["clip_coef"], ent=mu["ent_coef"], vf=mu["vf_coef"], mgn=mu["max_grad_norm"],
                   eps=mu["adam_eps"], options=opts)
    ag.load_params(p)
    O_, A = meta["O"], meta["A"]
    ag.buffer(ppo_amd.BUF_OBS, (1, M, O_)).upload(d["x"].reshape(1, M, O_))
    ag.buffer(ppo_amd.BUF_ACTIONS, (1, M, A)).upload(d["action"].reshape(1, M, A))
    for buf, key in ((ppo_amd.BUF_LOGPROBS, "old_logp"), (ppo_amd.BUF_ADVANTAGES, "adv"),
                     (ppo_amd.BUF_RETURNS, "ret"), (ppo_amd.BUF_VALUES, "old_v")):
        ag.buffer(buf, (1, M)).upload(d[key].reshape(1, M))
    perm = DeviceArray.from_numpy(np.arange(M, dtype=np.int32))
    st = ag.update(mu["lr"], perms=perm)
    g = ag.last_grad()
    assert rel(g, d["grad_raw"]) < 2e-4, rel(g, d["grad_raw"])
    L = ag.layout
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if L.t_grad[t]:
            assert rel(g[o:o + n], d["grad_raw"][o:o + n]) < 2e-3, (t, rel(g[o:o + n], d["grad_raw"][o:o + n]))
    np.testing.assert_allclose([st["pg_loss"], st["v_loss"], st["entropy"], st["old_approx_kl"], st["approx_kl"],
                                st["clipfrac"]], d["stats"][:6], rtol=2e-4, atol=2e-5)
    np.testing.assert_allclose(st["grad_norm"], d["total_norm"][0], rtol=2e-4)
    np.testing.assert_allclose(ag.params(), d["params_step1"], rtol=0, atol=2e-6)
    ag.update(mu["lr"], perms=perm)
    ag.update(mu["lr"], perms=perm)
    np.testing.assert_allclose(ag.params(), d["params_step3"], rtol=0, atol=6e-6)
    ag.close()


@pytest.mark.parametrize("T", [1, 7, 33])
def test_gae_ragged_bit_exact_vs_golden(T):
    _, d = load_case(f"gae_t{T}")
    E = d["rewards"].shape[1]
    ag = agent_for({"kind": 0, "O": 17, "A": 6, "H": 64}, E, T=T)
    for buf, key in ((ppo_amd.BUF_REWARDS, "rewards"), (ppo_amd.BUF_VALUES, "values"), (ppo_amd.BUF_DONES, "dones")):
        ag.buffer(buf, (T, E)).upload(d[key])
    ag.gae_from_values(DeviceArray.from_numpy(d["next_value"]), DeviceArray.from_numpy(d["next_done"]))
    np.testing.assert_array_equal(ag.buffer(ppo_amd.BUF_ADVANTAGES, (T, E)).numpy(), d["advantages"])
    np.testing.assert_array_equal(ag.buffer(ppo_amd.BUF_RETURNS, (T, E)).numpy(), d["returns"])
    ag.close()


def test_gae_long_bit_exact_vs_golden():
    """cfg2's T=2048 at E=1024: 64 load chunks per env; compared through per-column FNV hashes."""
    meta, d = load_case("gae_long")
    T, E = meta["T"], meta["E"]
    r, v, dn, nv, nd = gae_long_inputs(T, E)
    # gae=auto runs the scan at T >= 512 (test_gae_scan_vs_golden); the serial kernel is the bit-exact one
    ag = agent_for({"kind": 0, "O": 17, "A": 6, "H": 64}, E, T=T, options="gae=serial")
    ag.buffer(ppo_amd.BUF_REWARDS, (T, E)).upload(r)
    ag.buffer(ppo_amd.BUF_VALUES, (T, E)).upload(v)
    ag.buffer(ppo_amd.BUF_DONES, (T, E)).upload(dn)
    ag.gae_from_values(DeviceArray.from_numpy(nv), DeviceArray.from_numpy(nd))
    adv = ag.buffer(ppo_amd.BUF_ADVANTAGES, (T, E)).numpy()
    ret = ag.buffer(ppo_amd.BUF_RETURNS, (T, E)).numpy()
    np.testing.assert_array_equal(adv[:, :8], d["adv_cols8"])
    np.testing.assert_array_equal(column_fnv(adv), d["adv_fnv"])
    np.testing.assert_array_equal(column_fnv(ret), d["ret_fnv"])
    ag.close()


@pytest.mark.parametrize("case", ["gae", "gae_t1", "gae_t7", "gae_t33", "gae_long"])
def test_gae_scan_vs_golden(case):
    """k_gae_scan (gae=scan; gae=auto's choice from T = 512, i.e. cfg1 / cfg2's T = 2 048) against the
    LibTorch-replay golden vectors of the reference's serial recurrence (ppo:447-467): advantages and
    returns within rtol 1e-5 / atol 1e-5 (the composed incoming value of each 1/16 segment rounds
    differently from the serial chain; max |d| printed). gae_long (T = 2 048, E = 1 024) holds its
    golden as 8 full columns plus per-column FNV hashes: the 8 columns are compared directly and every
    column against the C oracle, which reproduces the hashes bit for bit (test_oracle_golden)."""
    meta, d = load_case(case)
    if case == "gae_long":
        T, E = meta["T"], meta["E"]
        r, v, dn, nv, nd = gae_long_inputs(T, E)
    else:
        r, v, dn, nv, nd = d["rewards"], d["values"], d["dones"], d["next_value"], d["next_done"]
        T, E = r.shape
    ag = agent_for({"kind": 0, "O": 17, "A": 6, "H": 64}, E, T=T, options="gae=scan")
    ag.buffer(ppo_amd.BUF_REWARDS, (T, E)).upload(r)
    ag.buffer(ppo_amd.BUF_VALUES, (T, E)).upload(v)
    ag.buffer(ppo_amd.BUF_DONES, (T, E)).upload(dn)
    ag.gae_from_values(DeviceArray.from_numpy(nv), DeviceArray.from_numpy(nd))
    adv = ag.buffer(ppo_amd.BUF_ADVANTAGES, (T, E)).numpy()
    ret = ag.buffer(ppo_amd.BUF_RETURNS, (T, E)).numpy()
    ag.close()
    if case == "gae_long":
        np.testing.assert_allclose(adv[:, :8], d["adv_cols8"], rtol=1e-5, atol=1e-5)
        ref_adv, ref_ret = O.gae(r, v, dn, nv, nd, 0.99, 0.95)
        assert (column_fnv(ref_adv) == d["adv_fnv"]).all() and (column_fnv(ref_ret) == d["ret_fnv"]).all()
    else:
        ref_adv, ref_ret = d["advantages"], d["returns"]
    print(f"\n{case} T={T} E={E}: max |adv scan - golden| {np.abs(adv - ref_adv).max():.2e}")
    np.testing.assert_allclose(adv, ref_adv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret, ref_ret, rtol=1e-5, atol=1e-5)
