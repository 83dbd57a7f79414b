"""LibTorch checkpoint interop: include/ppo_pth.h against archives the reference's
LibTorch wrote.

Fixtures tests/golden/pth_{ppo,ac}/ come from oracle/ref_harness.cpp ("pth_ppo" / "pth_ac"): the
reference agents (O=5, A=2, H=16) after two Adam steps, saved with torch::save(agent) /
torch::save(optimizer) exactly as save_state does (src/ppo_continuous_action.cpp:173-180), plus
their flat parameters and Adam moments. Checked here, on CPU (no GPU call):
  * reading: torch::save archives -> flat vectors, bit-exact;
  * writing: our model archive's data.pkl, class files and tensor data are byte-identical to
    torch::save's; archives load in PyTorch (torch.jit.load) with the same values;
  * the reverse direction through LibTorch itself: `ref_harness --pth-load` torch::loads our
    model + optimizer archives into the reference agent / Adam (skipped where the harness is not
    built, e.g. on the GPU box);
  * error behaviour: shape mismatch / missing parameter / wrong parameter count raise.
"""
import json
import os
import subprocess
import zipfile

import numpy as np
import pytest

try:  # torch before libppo_hip: torch bundles its own HIP runtime, which must be the first loaded
    import torch
except ImportError:  # pragma: no cover
    torch = None

import ppo_amd as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
CASES = [(P.PPO_NET_TANH_NORMAL, "pth_ppo"), (P.PPO_NET_LN_BETA, "pth_ac")]


def _gold(case, name):
    return np.fromfile(os.path.join(GOLD, case, name + ".f32"), np.float32)


def _entries(path):
    """archive entries without the top-level folder (torch::save names it after the file stem)"""
    z = zipfile.ZipFile(path)
    return {n.split("/", 1)[1]: z.read(n) for n in z.namelist()}


@pytest.mark.parametrize("kind,case", CASES)
def test_read_reference_archives(kind, case):
    L = P.agent_layout(kind, 5, 2, 16)
    p = P.load_agent_pth(L, os.path.join(GOLD, case, "model.pth"))
    assert np.array_equal(p, _gold(case, "params"))
    m, v, step, lr, eps = P.load_adam_pth(L, os.path.join(GOLD, case, "optimizer.pth"))
    assert np.array_equal(m, _gold(case, "adam_m")) and np.array_equal(v, _gold(case, "adam_v"))
    assert step == 2 and lr == pytest.approx(2.5e-4, rel=1e-12) and eps == pytest.approx(1e-5, rel=1e-12)


@pytest.mark.parametrize("kind,case", CASES)
def test_model_archive_byte_identical(kind, case, tmp_path):
    L = P.agent_layout(kind, 5, 2, 16)
    out = tmp_path / "model.pth"
    P.save_agent_pth(L, _gold(case, "params"), out)
    ref, ours = _entries(os.path.join(GOLD, case, "model.pth")), _entries(out)
    assert set(ref) == set(ours)
    for name in ref:
        if name == ".data/serialization_id":  # torch::save draws it at random
            assert len(ours[name]) == len(ref[name])
            continue
        assert ours[name] == ref[name], name
    # stored entries, data 64-byte aligned (mmap-able like torch::save's)
    z = zipfile.ZipFile(out)
    for info in z.infolist():
        assert info.compress_type == zipfile.ZIP_STORED
        if "/data/" in info.filename:
            raw = open(out, "rb").read()
            hdr = info.header_offset
            nlen, xlen = np.frombuffer(raw[hdr + 26:hdr + 30], np.uint16)
            assert (hdr + 30 + nlen + xlen) % 64 == 0


@pytest.mark.parametrize("kind,case", CASES)
def test_archives_load_in_pytorch(kind, case, tmp_path):
    if torch is None:
        pytest.skip("torch not importable")
    L = P.agent_layout(kind, 5, 2, 16)
    params = _gold(case, "params")
    P.save_agent_pth(L, params, tmp_path / "model.pth")
    mod = torch.jit.load(str(tmp_path / "model.pth"))
    meta = json.load(open(os.path.join(GOLD, "manifest.json")))[case]["meta"]
    names = [n for n, _, _ in meta["params"]]
    got = dict(mod.named_parameters())
    assert list(got) == names  # named_parameters() order = the flat order
    flat = np.concatenate([got[n].detach().numpy().reshape(-1) for n in names])
    assert np.array_equal(flat, params)
    for n, _, grad in meta["params"]:
        assert got[n].requires_grad == bool(grad), n
    # optimizer archive: state per trainable parameter, keyed through param_groups/0/params/<i>
    m, v = _gold(case, "adam_m"), _gold(case, "adam_v")
    P.save_adam_pth(L, m, v, 2, 2.5e-4, 1e-5, tmp_path / "optimizer.pth")
    opt = torch.jit.load(str(tmp_path / "optimizer.pth"))
    g = getattr(opt.param_groups, "param_groups/0")
    assert int(getattr(g, "params/size")) == L.ntensors
    assert g.options.lr == 2.5e-4 and g.options.eps == 1e-5 and tuple(g.options.betas) == (0.9, 0.999)
    for t in range(L.ntensors):
        key = getattr(g, f"params/{t}")
        o, n = L.t_off[t], L.t_len[t]
        if not L.t_grad[t]:
            assert not hasattr(opt.state, key)
            continue
        st = getattr(opt.state, key)
        assert st.step == 2
        assert np.array_equal(st.exp_avg.numpy().reshape(-1), m[o:o + n])
        assert np.array_equal(st.exp_avg_sq.numpy().reshape(-1), v[o:o + n])


@pytest.mark.parametrize("kind,case", CASES)
def test_libtorch_loads_our_archives(kind, case, tmp_path):
    if not os.path.exists(HARNESS):
        pytest.skip("oracle/_ref/ref_harness not built (needs /root/reference + LibTorch)")
    L = P.agent_layout(kind, 5, 2, 16)
    rng = np.random.default_rng(kind + 7)
    params = rng.standard_normal(L.P).astype(np.float32)
    m = rng.standard_normal(L.P).astype(np.float32)
    v = np.abs(rng.standard_normal(L.P)).astype(np.float32)
    for t in range(L.ntensors):  # no state for parameters without gradient
        if not L.t_grad[t]:
            m[L.t_off[t]:L.t_off[t] + L.t_len[t]] = 0
            v[L.t_off[t]:L.t_off[t] + L.t_len[t]] = 0
    P.save_agent_pth(L, params, tmp_path / "model_final.pth")
    P.save_adam_pth(L, m, v, 37, 1.25e-4, 1e-5, tmp_path / "optimizer_final.pth")
    out = tmp_path / "loaded"
    subprocess.run([HARNESS, "--pth-load", "ppo" if kind == 0 else "ac", "5", "2", "16",
                    str(tmp_path / "model_final.pth"), str(tmp_path / "optimizer_final.pth"), str(out)],
                   check=True, timeout=120)
    meta = json.load(open(out / "manifest.json"))["loaded"]["meta"]
    assert meta["step"] == 37 and meta["lr"] == pytest.approx(1.25e-4) and meta["eps"] == pytest.approx(1e-5)
    assert np.array_equal(np.fromfile(out / "loaded" / "params.f32", np.float32), params)
    assert np.array_equal(np.fromfile(out / "loaded" / "adam_m.f32", np.float32), m)
    assert np.array_equal(np.fromfile(out / "loaded" / "adam_v.f32", np.float32), v)


def test_carla_archive_roundtrip(tmp_path):
    if torch is None:
        pytest.skip("torch not importable")
    L = P.carla_layout()
    params = np.random.default_rng(3).standard_normal(L.P).astype(np.float32)
    P.save_carla_pth(L, params, tmp_path / "model_0.pth")
    assert np.array_equal(P.load_carla_pth(L, tmp_path / "model_0.pth"), params)
    mod = torch.jit.load(str(tmp_path / "model_0.pth"))
    sd = dict(mod.named_parameters())
    assert list(sd)[:4] == ["action_space_high", "action_space_low", "cnn.0.weight", "cnn.0.bias"]
    assert tuple(sd["cnn.0.weight"].shape) == (8, 15, 5, 5) and tuple(sd["linear.0.weight"].shape) == (512, 1280)
    assert len(sd) == L.ntensors
    flat = np.concatenate([t.detach().numpy().reshape(-1) for t in sd.values()])
    assert np.array_equal(flat, params)
    assert len(list(mod.cnn.children())) == 12  # Conv2d / ReLU pairs, as carla_model.h's roach encoder


def test_load_errors(tmp_path):
    Lp = P.agent_layout(P.PPO_NET_TANH_NORMAL, 5, 2, 16)
    with pytest.raises(P.PPOError, match="shape mismatch"):
        P.load_agent_pth(P.agent_layout(P.PPO_NET_TANH_NORMAL, 5, 2, 32), os.path.join(GOLD, "pth_ppo", "model.pth"))
    with pytest.raises(P.PPOError, match="no parameter|no module"):
        P.load_agent_pth(P.agent_layout(P.PPO_NET_LN_BETA, 5, 2, 16), os.path.join(GOLD, "pth_ppo", "model.pth"))
    with pytest.raises(P.PPOError, match="parameters"):
        P.load_adam_pth(P.agent_layout(P.PPO_NET_LN_BETA, 5, 2, 16), os.path.join(GOLD, "pth_ppo", "optimizer.pth"))
    with pytest.raises(P.PPOError, match="cannot open"):
        P.load_agent_pth(Lp, tmp_path / "missing.pth")
    (tmp_path / "junk.pth").write_bytes(b"not a zip archive at all")
    with pytest.raises(P.PPOError, match="zip"):
        P.load_agent_pth(Lp, tmp_path / "junk.pth")
    with pytest.raises(P.PPOError):
        P.carla_layout(15, 100, 100)  # n_flatten != 256 * 2 * 2
