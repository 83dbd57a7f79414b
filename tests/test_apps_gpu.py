"""The two drop-in trainer executables (ppo.cpp_amd/bin/{ppo,ac_ppo}_continuous_action, same flags
as src/ppo_continuous_action.cpp / src/ac_ppo_continuous_action.cpp) run end to end on the GPU.

The AC-PPO run with host envs (gymcpp SeqVectorEnv per env, async collection groups on HIP
streams) and with the device-resident env must end with bit-identical weights: the host env is
bit-identical to the device env (tests/test_host_env.py), actions come from counter-based Philox
draws that do not depend on how envs are grouped, and the update path is shared."""
import os
import subprocess

import numpy as np
import pytest

import ppo_amd as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ppo.cpp_amd")
BIN = os.path.join(PKG, "bin")
MODELS = os.path.join(PKG, "models")


def _exe(name):
    path = os.path.join(BIN, name)
    if not os.path.exists(path):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    return path


def _run(args, timeout=240):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout


@pytest.mark.gpu
def test_ppo_cli_runs():
    out = _run([_exe("ppo_continuous_action"), "--env_id", "SyntheticCheetah-v0", "--num_envs", "8",
                "--num_steps", "64", "--total_timesteps", str(8 * 64 * 3), "--num_eval_runs", "1",
                "--exp_name_stem", "t_ppo_cli", "--seed", "3"])
    assert "SPS:" in out
    # model_final.pth / optimizer_final.pth: LibTorch archives of the reference agent (ppo:587)
    L = P.agent_layout(P.PPO_NET_TANH_NORMAL, 17, 6, 64)
    p = P.load_agent_pth(L, os.path.join(MODELS, "t_ppo_cli_3", "model_final.pth"))
    assert p.size == L.P and np.isfinite(p).all()
    m, v, step, lr, eps = P.load_adam_pth(L, os.path.join(MODELS, "t_ppo_cli_3", "optimizer_final.pth"))
    assert step == 3 * 10 * 32 and np.isfinite(m).all() and (v >= 0).all() and eps == pytest.approx(1e-5)
    latest = [f for f in os.listdir(os.path.join(MODELS, "t_ppo_cli_3")) if f.startswith("model_latest_")]
    assert len(latest) == 1 and latest[0].endswith(".pth")  # older ones cleaned up (ppo:548-556)
    # the reference's TensorBoard event file (ppo:281), one record per scalar of the JSON-lines log
    ev = open(os.path.join(MODELS, "t_ppo_cli_3", "tfevents_logs.pb"), "rb").read()
    n_lines = len(open(os.path.join(MODELS, "t_ppo_cli_3", "scalars.jsonl")).read().splitlines())
    pos, records = 0, 0
    while pos < len(ev):
        (n,) = np.frombuffer(ev[pos:pos + 8], np.uint64)
        pos += 12 + int(n) + 4
        records += 1
    assert pos == len(ev) and records == n_lines > 0


@pytest.mark.gpu
@pytest.mark.parametrize("E,T,groups,host_us", [(64, 16, "5", "0"), (4096, 8, "0", "0"), (512, 8, "0", "2")])
def test_ac_cli_host_equals_device_env(E, T, groups, host_us):
    """Host envs in async collection groups (5 groups; the default two per host thread at cfg3's
    E = 4096; with a per-step host cost) vs the device env: bit-identical weights."""
    tag = f"{E}_{T}_{groups}_{host_us}".replace(".", "p")
    common = ["--num_envs", str(E), "--num_steps", str(T), "--total_timesteps", str(E * T * 2), "--seed", "4",
              "--num_eval_runs", "1"]
    out = _run([_exe("ac_ppo_continuous_action"), "--env_id", "SyntheticCheetah-v0", "--env_backend", "host",
                "--num_collect_groups", groups, "--host_step_us", host_us, "--exp_name_stem", f"t_ac_host{tag}"] + common)
    assert "collection groups: " in out
    _run([_exe("ac_ppo_continuous_action"), "--env_id", "SyntheticCheetah-v0", "--env_backend", "device",
          "--exp_name_stem", f"t_ac_dev{tag}"] + common)
    L = P.agent_layout(P.PPO_NET_LN_BETA, 17, 6, 256)
    a = P.load_agent_pth(L, os.path.join(MODELS, f"t_ac_host{tag}_4", "model_final.pth"))
    b = P.load_agent_pth(L, os.path.join(MODELS, f"t_ac_dev{tag}_4", "model_final.pth"))
    assert a.size == b.size and a.size > 146189
    np.testing.assert_array_equal(a, b)


def _free_port_pair():
    import socket
    for _ in range(50):
        with socket.socket() as s0:
            s0.bind(("127.0.0.1", 0))
            p = s0.getsockname()[1]
        try:
            with socket.socket() as s1:
                s1.bind(("127.0.0.1", p + 1))
            return p
        except OSError:
            continue
    raise RuntimeError("no free port pair")


@pytest.mark.gpu
def test_ac_cli_dd_ppo_preemption_with_a_straggler_group():
    """DD-PPO preemption (ac:568-583, :680-693, :803-810) through the drop-in CLI: 4 collection groups,
    the last one 200 us per env step slower. The other three finish all 64 steps while the straggler
    is still early, so once it is past dd_ppo_min_perc (0.25 x 64 = 16 steps) it sees 3 of 4 groups
    done (> 0.6) and stops after step 17: both iterations train on 17 steps per env (the step at
    which it stops is stored but not trained on, as in the reference), the batch padded by repeating
    the permutation (the index rule itself: test_gpu_ddppo.py)."""
    port = _free_port_pair()
    out = _run([_exe("ac_ppo_continuous_action"), "--env_id", "SyntheticCheetah-v0", "--env_backend", "host",
                "--num_envs", "64", "--num_steps", "64", "--total_timesteps", str(64 * 64 * 2), "--seed", "6",
                "--num_eval_runs", "1", "--num_collect_groups", "4", "--straggler_us", "200",
                "--use_dd_ppo_preempt", "1", "--dd_ppo_min_perc", "0.25", "--dd_ppo_preempt_threshold", "0.6",
                "--rdzv_addr", "127.0.0.1", "--tcp_store_port", str(port), "--exp_name_stem", "t_ac_ddppo"])
    assert out.count("dd_ppo: rank 0 trains on 17 of 64 steps per env (preempted)") == 2, out[-3000:]
    L = P.agent_layout(P.PPO_NET_LN_BETA, 17, 6, 256)
    p = P.load_agent_pth(L, os.path.join(MODELS, "t_ac_ddppo_6", "model_final.pth"))
    assert np.isfinite(p).all()
    # without preemption the same run trains on all 64 steps
    out = _run([_exe("ac_ppo_continuous_action"), "--env_id", "SyntheticCheetah-v0", "--env_backend", "host",
                "--num_envs", "64", "--num_steps", "64", "--total_timesteps", str(64 * 64 * 2), "--seed", "6",
                "--num_eval_runs", "1", "--num_collect_groups", "4", "--exp_name_stem", "t_ac_noddppo"])
    assert "dd_ppo:" not in out


@pytest.mark.gpu
def test_ac_cli_estimate_mean_std_host_equals_device():
    """--estimate_mean_std (ac:663, :954-963): mean and population std of env 0's observations over the
    run, printed at the end; the host and the device env give the same trajectories, so the same numbers."""
    outs = []
    for backend in ("host", "device"):
        out = _run([_exe("ac_ppo_continuous_action"), "--env_id", "SyntheticCheetah-v0", "--env_backend", backend,
                    "--num_envs", "8", "--num_steps", "16", "--total_timesteps", str(8 * 16 * 2), "--seed", "2",
                    "--num_eval_runs", "1", "--estimate_mean_std", "1", "--exp_name_stem", f"t_ac_ems_{backend}"])
        tail = out[out.index("Mean obs:"):]
        tail = tail[:tail.index("]", tail.index("Std obs:"))]
        vals = [float(x) for x in tail.split() if x.replace(".", "").replace("-", "").replace("e", "").isdigit()]
        outs.append(vals)
    assert len(outs[0]) == 34 and outs[0] == outs[1]
    assert all(v >= 0 for v in outs[0][17:])


@pytest.mark.gpu
def test_ppo_cli_host_equals_device_env():
    """ppo_continuous_action with host envs (ParVectorEnv of gymcpp::make_env: the wrapper chain of
    ppo:41-49 on the CPU) and with --env_backend device (the same chain fused into the device env's
    kernels) ends with bit-identical weights over 3 iterations with autoresets: the device chain
    reproduces the host chain bit for bit inside the full training loop."""
    common = ["--env_id", "SyntheticCheetah-v0", "--num_envs", "4", "--num_steps", "400", "--num_minibatches", "4",
              "--update_epochs", "2", "--total_timesteps", str(4 * 400 * 3), "--seed", "5", "--num_eval_runs", "1"]
    _run([_exe("ppo_continuous_action"), "--env_backend", "host", "--exp_name_stem", "t_ppo_host"] + common)
    _run([_exe("ppo_continuous_action"), "--env_backend", "device", "--exp_name_stem", "t_ppo_dev"] + common)
    L = P.agent_layout(P.PPO_NET_TANH_NORMAL, 17, 6, 64)
    a = P.load_agent_pth(L, os.path.join(MODELS, "t_ppo_host_5", "model_final.pth"))
    b = P.load_agent_pth(L, os.path.join(MODELS, "t_ppo_dev_5", "model_final.pth"))
    np.testing.assert_array_equal(a, b)


@pytest.mark.gpu
def test_ppo_cli_cfg2_humanoid_device_env():
    """BASELINE cfg2 through the drop-in executable: Humanoid-v4 shapes (O=376, A=17, actions in
    [-0.4, 0.4]), num_envs=1024, the reference defaults otherwise (num_steps 2048, 32 minibatches,
    10 epochs), the wrapper chain on the device; two iterations and the final evaluation."""
    E, T = 1024, 2048
    out = _run([_exe("ppo_continuous_action"), "--env_id", "Humanoid-v4", "--env_backend", "device", "--num_envs",
                str(E), "--total_timesteps", str(E * T * 2), "--exp_name_stem", "t_ppo_cfg2", "--seed", "1"])
    assert out.count("SPS:") == 2 and "Average evaluation return=" in out
    L = P.agent_layout(P.PPO_NET_TANH_NORMAL, 376, 17, 64)
    p = P.load_agent_pth(L, os.path.join(MODELS, "t_ppo_cfg2_1", "model_final.pth"))
    assert p.size == L.P and np.isfinite(p).all()


@pytest.mark.gpu
def test_ac_cli_ant_device_env():
    """cfg4's agent shape (Ant-v5: O=105, A=8, the Ant observation normalisation table) on the device env
    through ac_ppo_continuous_action."""
    out = _run([_exe("ac_ppo_continuous_action"), "--env_id", "Ant-v5", "--env_backend", "device", "--num_envs", "256",
                "--num_steps", "32", "--total_timesteps", str(256 * 32 * 2), "--exp_name_stem", "t_ac_ant",
                "--num_eval_runs", "1"])
    assert out.count("SPS:") == 2
    L = P.agent_layout(P.PPO_NET_LN_BETA, 105, 8, 256)
    p = P.load_agent_pth(L, os.path.join(MODELS, "t_ac_ant_1", "model_final.pth"))
    assert np.isfinite(p).all()


def test_cli_flag_errors():
    """Flag parsing follows args.hxx: unknown flags / bad bool values fail with a message (no GPU)."""
    exe = _exe("ac_ppo_continuous_action")
    r = subprocess.run([exe, "--no_such_flag", "1"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "no_such_flag" in r.stderr
    r = subprocess.run([exe, "--norm_adv", "true"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "norm_adv" in r.stderr
    r = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--num_envs" in r.stdout


def tb_scalars(path):
    """(tag, step, simple_value) of every Summary.Value in a TFRecord event file (minimal protobuf
    reader: Event.step = field 2 varint, Event.summary = field 5, Summary.value = field 1,
    Value.tag = field 1, Value.simple_value = field 2 float)."""
    import struct

    def fields(buf):
        i = 0
        while i < len(buf):
            key, i = _varint(buf, i)
            f, wt = key >> 3, key & 7
            if wt == 0:
                v, i = _varint(buf, i)
            elif wt == 1:
                v, i = buf[i:i + 8], i + 8
            elif wt == 5:
                v, i = buf[i:i + 4], i + 4
            else:
                n, i = _varint(buf, i)
                v, i = buf[i:i + n], i + n
            yield f, v

    ev = open(path, "rb").read()
    out, pos = [], 0
    while pos < len(ev):
        (n,) = struct.unpack_from("<Q", ev, pos)
        rec = ev[pos + 12:pos + 12 + n]
        pos += 12 + n + 4
        step = 0
        for f, v in fields(rec):
            if f == 2:
                step = v
            elif f == 5:
                for sf, sv in fields(v):
                    if sf == 1:
                        tag, val = None, None
                        for vf, vv in fields(sv):
                            if vf == 1:
                                tag = vv.decode()
                            elif vf == 2:
                                val = struct.unpack("<f", vv)[0]
                        out.append((tag, step, val))
    return out


def _varint(b, i):
    r, s = 0, 0
    while True:
        c = b[i]
        i += 1
        r |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return r, i


@pytest.mark.gpu
@pytest.mark.parametrize("exe,lr0,E,T", [("ppo_continuous_action", 3e-4, 8, 64), ("ac_ppo_continuous_action", 2.5e-4, 16, 16)])
def test_lr_anneal_schedule_and_async_checkpoints(exe, lr0, E, T):
    """LR anneal (ppo:379-384, ac:634-639): lrnow = (1 - it / num_iterations) * lr0 in float32,
    read back from the charts/learning_rate scalars of the TensorBoard file; and the checkpoints
    written off the critical path: the last model_latest_*.pth (async snapshot after the last
    update) holds exactly the parameters of model_final.pth."""
    n_it = 5
    stem = f"t_lr_{exe[:3]}"
    extra = ["--env_backend", "device"] if exe.startswith("ac") else []
    _run([_exe(exe), "--env_id", "SyntheticCheetah-v0", "--num_envs", str(E), "--num_steps", str(T),
          "--total_timesteps", str(E * T * n_it), "--num_eval_runs", "1", "--exp_name_stem", stem, "--seed", "2"] + extra)
    d = os.path.join(MODELS, f"{stem}_2")
    tb = "tfevents_logs.pb" if exe.startswith("ppo") else "tfevents_logs_0.pb"
    lrs = [(s, v) for tag, s, v in tb_scalars(os.path.join(d, tb)) if tag == "charts/learning_rate"]
    assert len(lrs) == n_it
    want = [np.float32(np.float32(1.0) - np.float32(i) / np.float32(n_it)) * np.float32(lr0) for i in range(n_it)]
    np.testing.assert_array_equal(np.float32([v for _, v in lrs]), np.float32(want))
    assert [s for s, _ in lrs] == [E * T * (i + 1) for i in range(n_it)]
    kind = P.PPO_NET_TANH_NORMAL if exe.startswith("ppo") else P.PPO_NET_LN_BETA
    L = P.agent_layout(kind, 17, 6, 64 if kind == P.PPO_NET_TANH_NORMAL else 256)
    latest = sorted(f for f in os.listdir(d) if f.startswith("model_latest_"))
    assert latest == [f"model_latest_{n_it - 1:09d}.pth"]
    np.testing.assert_array_equal(P.load_agent_pth(L, os.path.join(d, latest[0])),
                                  P.load_agent_pth(L, os.path.join(d, "model_final.pth")))
    m, v, step, lr, eps = P.load_adam_pth(L, os.path.join(d, f"optimizer_latest_{n_it - 1:09d}.pth"))
    mf, vf, stepf, _, _ = P.load_adam_pth(L, os.path.join(d, "optimizer_final.pth"))
    assert step == stepf and np.array_equal(m, mf) and np.array_equal(v, vf)
    assert lr == pytest.approx(float(want[-1]), rel=1e-6)
