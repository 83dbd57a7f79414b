"""CPU-side checks of the C-ABI boundary: libppo_hip.so loads and exports every entry point
declared in include/*.h (no compute calls — there is no GPU here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip.so")


def declared_functions():
    names = []
    hdrs = sorted(h for h in os.listdir(os.path.join(ROOT, "include")) if h.endswith(".h"))
    assert {"ppo_hip.h", "ppo_synth_env.h", "ppo_env_wrappers.h", "ppo_carla.h", "ppo_pth.h"} <= set(hdrs)
    for h in hdrs:
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b((?:ppo|psyn|pwrap)_\w+)\s*\(", src, flags=re.M):
            if "static" not in m.group(0):  # header-only helpers (static inline layout initialisers)
                names.append(m.group(1))
    return sorted(set(names))


def test_headers_declare_the_boundary():
    names = declared_functions()
    for required in ("ppo_create", "ppo_get_action_and_value", "ppo_rollout_act", "ppo_compute_gae", "ppo_update",
                     "ppo_comm_init", "ppo_comm_info", "ppo_get_device", "psyn_step", "pwrap_step", "psyn_attach_wrappers",
                     "ppo_set_rollout_mode"):
        assert required in names


@pytest.mark.skipif(not os.path.exists(LIB), reason="libppo_hip.so not built (run __graft_entry__.build())")
def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


@pytest.mark.skipif(not os.path.exists(LIB), reason="libppo_hip.so not built")
def test_python_binding_covers_every_symbol():
    import ppo_amd
    bound = {n for n, _, _ in ppo_amd.SYMBOLS}
    assert set(declared_functions()) <= bound
    lib = ppo_amd.lib()
    assert b"gfx950" in lib.ppo_version()


def test_layout_header_matches_python_restatement():
    """include/ppo_layout.h offsets (compiled C) == tests/oracle_lib.layout_init (restated)."""
    import subprocess
    import tempfile
    import oracle_lib as O
    src = r'''
#include <stdio.h>
#include "ppo_layout.h"
int main(void) {
  int cases[][4] = {{0,17,6,64},{1,17,6,256},{0,376,17,64},{1,105,8,256}};
  for (int c = 0; c < 4; ++c) {
    ppo_layout L; ppo_layout_init(&L, cases[c][0], cases[c][1], cases[c][2], cases[c][3]);
    printf("%ld %ld %d", L.P, L.train_begin, L.ntensors);
    for (int t = 0; t < L.ntensors; ++t) printf(" %ld:%ld:%d", L.t_off[t], L.t_len[t], L.t_grad[t]);
    printf("\n");
  }
  return 0;
}'''
    with tempfile.TemporaryDirectory() as d:
        cpath = os.path.join(d, "l.c")
        open(cpath, "w").write(src)
        exe = os.path.join(d, "l")
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), cpath, "-o", exe])
        lines = subprocess.check_output([exe]).decode().strip().splitlines()
    for line, (k, o, a, h) in zip(lines, [(0, 17, 6, 64), (1, 17, 6, 256), (0, 376, 17, 64), (1, 105, 8, 256)]):
        L = O.layout_init(k, o, a, h)
        parts = line.split()
        assert int(parts[0]) == L.P and int(parts[1]) == L.train_begin and int(parts[2]) == L.ntensors
        for t, tok in enumerate(parts[3:]):
            off, ln, gr = map(int, tok.split(":"))
            assert (off, ln, gr) == (L.t_off[t], L.t_len[t], L.t_grad[t])
    # the AC HalfCheetah agent has the survey's 146,189 trainable parameters
    L = O.layout_init(1, 17, 6, 256)
    assert L.P - L.train_begin == 146189
    assert O.layout_init(0, 17, 6, 64).P == 11085



BAD_CONFIGS = [
    ("num_envs", 0, "sizes must be positive"),            # empty rollout
    ("num_steps", -1, "sizes must be positive"),
    ("num_minibatches", 0, "sizes must be positive"),
    ("update_epochs", 0, "sizes must be positive"),
    ("num_minibatches", 7, "must divide by num_minibatches"),  # ragged minibatches (ac:407 asserts it too)
    ("num_envs", 1 << 24, "batch too large"),            # T*E rows beyond a 31-bit index
    ("hidden", 128, "hidden must be 64 or 256"),
    ("act_dim", 0, "bad net kind / dims"),
    ("net_kind", 5, "bad net kind / dims"),
]


@pytest.mark.skipif(not os.path.exists(LIB), reason="libppo_hip.so not built")
def test_create_rejects_bad_configs():
    """ppo_create validates its configuration before touching the GPU: every bad shape is refused
    with a message through ppo_last_error and no context is returned (the reference asserts the
    same preconditions, ac:399-407). Run in a fresh interpreter: ppo_amd loads torch first, as
    every consumer of the library must (an earlier test here maps the library without torch)."""
    import json
    import subprocess
    import sys
    script = r'''
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
import ppo_amd
lib = ppo_amd.lib()
out = []
for field, value, _ in json.loads(sys.argv[2]):
    cfg = ppo_amd.HipConfig(net_kind=1, obs_dim=17, act_dim=6, hidden=256, num_envs=4096, num_steps=128,
                            num_minibatches=4, update_epochs=4)
    setattr(cfg, field, value)
    ctx = ctypes.c_void_p()
    rc = lib.ppo_create(ctypes.byref(cfg), 0, ctypes.byref(ctx))
    out.append([rc, bool(ctx.value), lib.ppo_last_error().decode()])
print(json.dumps(out))
'''
    res = subprocess.run([sys.executable, "-c", script, os.path.join(ROOT, "ppo.cpp_amd"), json.dumps(BAD_CONFIGS)],
                         capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    got = json.loads(res.stdout.strip().splitlines()[-1])
    for (field, value, message), (rc, has_ctx, err) in zip(BAD_CONFIGS, got):
        assert rc != 0 and not has_ctx, (field, value)
        assert message in err, (field, value, err)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libppo_hip.so not built")
def test_create_ex_rejects_unknown_options():
    """ppo_create_ex / ppo_carla_create_ex parse their kernel-selection options before touching the
    GPU: an unknown key or value is refused with a message and no context."""
    import json
    import subprocess
    import sys
    script = r'''
import ctypes, json, sys
sys.path.insert(0, sys.argv[1])
import ppo_amd
lib = ppo_amd.lib()
out = []
for opt in ("upd_kernel=fast", "act_kernel=3", "bogus=1", "dw_fused", "rollout=sometimes", "dw_dma=2",
            "dw_rows=24", "dw_rows=0", "dw_rows=x", "dw_rows=99999999999", "dw_slices=3", "update_graph=2", "gradnorm=x",
            "upd2_split=1", "rollout_kernel=fast", "upd_mfma=8", "upd_mfma=bx9", "gae=parallel", "dw_mfma=bf16", "dw_mfma=x9"):
    cfg = ppo_amd.HipConfig(net_kind=1, obs_dim=17, act_dim=6, hidden=256, num_envs=64, num_steps=8,
                            num_minibatches=1, update_epochs=1)
    ctx = ctypes.c_void_p()
    rc = lib.ppo_create_ex(ctypes.byref(cfg), 0, opt.encode(), ctypes.byref(ctx))
    out.append([rc, bool(ctx.value), lib.ppo_last_error().decode()])
for opt in ("tail=coop", "conv1=staged,tail=", "conv1=fast", "conv1_mfma=bx9", "conv_dgrad=fast", "conv_wgrad=quad", "conv_fwd=x", "deep_dgrad=dense"):  # the CaRL agent's options
    cfg = ppo_amd.CarlaConfig(15, 192, 192, 8, 3, 2, 1.0, 32, 7, 0)
    ctx = ctypes.c_void_p()
    rc = lib.ppo_carla_create_ex(ctypes.byref(cfg), 0, opt.encode(), ctypes.byref(ctx))
    out.append([rc, bool(ctx.value), lib.ppo_last_error().decode()])
print(json.dumps(out))
'''
    res = subprocess.run([sys.executable, "-c", script, os.path.join(ROOT, "ppo.cpp_amd")], capture_output=True,
                         text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    for rc, has_ctx, err in json.loads(res.stdout.strip().splitlines()[-1]):
        assert rc != 0 and not has_ctx and ("ppo_create_ex" in err or "ppo_carla_create_ex" in err), err


@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "ppo.cpp_amd", "bin", "ac_ppo_continuous_action")),
                    reason="CLI not built")
def test_ac_cli_refuses_a_rank_without_a_gpu_id(tmp_path):
    """The reference picks its GPU as gpu_ids.at(local_rank) (ac:447-448 / :459-460), which throws
    for a rank without an entry; the drop-in CLI refuses such a rank with a message and exit code 2
    before any HIP call (so this runs without a GPU), instead of wrapping onto another rank's GPU."""
    import subprocess
    exe = os.path.join(ROOT, "ppo.cpp_amd", "bin", "ac_ppo_continuous_action")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "OMPI_COMM_WORLD_RANK",
                                                             "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK")}
    env["LOCAL_RANK"] = "1"
    r = subprocess.run([exe, "--env_backend", "device", "--total_timesteps", "1024", "--exp_name_stem", "refuse"],
                       capture_output=True, text=True, timeout=60, env=env, cwd=tmp_path)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "local rank 1 has no entry in --gpu_ids" in r.stderr


def test_ac_cli_refuses_dd_ppo_on_the_device_env(tmp_path):
    """DD-PPO preemption stops per-env collection threads early (ac:680-689); the device-resident
    rollout has none, so the CLI refuses the combination before any HIP call (exit 1)."""
    import subprocess
    exe = os.path.join(ROOT, "ppo.cpp_amd", "bin", "ac_ppo_continuous_action")
    r = subprocess.run([exe, "--env_backend", "device", "--use_dd_ppo_preempt", "1", "--total_timesteps", "1024",
                        "--exp_name_stem", "refuse_dd"], capture_output=True, text=True, timeout=60, cwd=tmp_path)
    assert r.returncode == 1, (r.returncode, r.stdout, r.stderr)
    assert "use_dd_ppo_preempt needs host envs" in r.stderr


def test_ac_cli_flags_of_round_5(tmp_path):
    """The AC CLI lists the collection flags (host cost per env step, straggler cost, group count with
    its automatic default) and estimate_mean_std in its --help, as args.hxx prints flags."""
    import subprocess
    exe = os.path.join(ROOT, "ppo.cpp_amd", "bin", "ac_ppo_continuous_action")
    r = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60, cwd=tmp_path)
    assert r.returncode == 0
    for flag in ("host_step_us", "straggler_us", "num_collect_groups", "estimate_mean_std", "use_dd_ppo_preempt"):
        assert flag in r.stdout, flag
