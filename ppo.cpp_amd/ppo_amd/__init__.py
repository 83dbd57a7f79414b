"""ppo_amd — Python host mirror of the MI355X-native PPO hot path (ctypes over libppo_hip.so).

The product is the C-ABI library built from ppo.cpp_amd/csrc (hand-written gfx950 kernels + the
C++ runtime). This module only binds it: no compute happens in Python and there is no CPU
fallback — if the HIP library is missing, importing it raises.

Mirrors of the reference interface (autonomousvision/ppo.cpp):
  * PPOConfig / ACPPOConfig  — GlobalConfig of src/ppo_continuous_action.cpp:51-118 and
                               src/ac_ppo_continuous_action.cpp:55-148 (same names and defaults)
  * Agent                    — AgentImpl::get_action_and_value / get_value
  * Trainer                  — the inline rollout -> GAE -> update loop of main()
  * Comm                     — torchfort::Comm (include/distributed.h:41-60) on RCCL
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

# One HIP runtime per process. torch bundles its own libamdhip64 and, if libppo_hip.so (linked
# against /opt/rocm's) is loaded first, `import torch` maps a second runtime next to it and the two
# tear each other down at exit (free(): invalid pointer). Importing torch first makes libppo_hip.so
# bind to the runtime already mapped (same soname), so processes that also use torch.distributed
# (bench.py --gpus N, the gloo tests) run on one runtime.
try:
    import torch  # noqa: F401
except ImportError:  # torch is plumbing only; the library works without it
    torch = None

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("PPO_HIP_LIB") or os.path.join(PKG_ROOT, "lib", "libppo_hip.so")  # override: diagnostics

PPO_NET_TANH_NORMAL = 0
PPO_NET_LN_BETA = 1
PPO_SAMPLE, PPO_MEAN, PPO_GIVEN = 0, 1, 2
(BUF_OBS, BUF_ACTIONS, BUF_LOGPROBS, BUF_REWARDS, BUF_DONES, BUF_VALUES, BUF_ADVANTAGES,
 BUF_RETURNS) = range(8)
MAX_T = 32


class PPOError(RuntimeError):
    pass


# int (*ppo_host_allreduce_fn)(float* host_buf, long n, int average, void* user)  (include/ppo_hip.h)
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_float), C.c_long, C.c_int, C.c_void_p)


class HipConfig(C.Structure):
    _fields_ = [("net_kind", C.c_int), ("obs_dim", C.c_int), ("act_dim", C.c_int), ("hidden", C.c_int),
                ("num_envs", C.c_int), ("num_steps", C.c_int), ("num_minibatches", C.c_int),
                ("update_epochs", C.c_int), ("gamma", C.c_float), ("gae_lambda", C.c_float),
                ("clip_coef", C.c_float), ("ent_coef", C.c_float), ("vf_coef", C.c_float),
                ("max_grad_norm", C.c_float), ("adam_eps", C.c_float), ("norm_adv", C.c_int),
                ("clip_vloss", C.c_int), ("seed", C.c_uint64), ("rank", C.c_int), ("world_size", C.c_int)]


class UpdateStats(C.Structure):
    _fields_ = [("pg_loss", C.c_float), ("v_loss", C.c_float), ("entropy", C.c_float),
                ("old_approx_kl", C.c_float), ("approx_kl", C.c_float), ("clipfrac", C.c_float),
                ("grad_norm", C.c_float), ("minibatches", C.c_int)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Layout(C.Structure):
    _fields_ = [("kind", C.c_int), ("O", C.c_int), ("A", C.c_int), ("H", C.c_int),
                ("P", C.c_long), ("train_begin", C.c_long),
                ("hi", C.c_long), ("lo", C.c_long), ("omean", C.c_long), ("ostd", C.c_long),
                ("logstd", C.c_long), ("critic", C.c_long * 8), ("actor", C.c_long * 8),
                ("cW3", C.c_long), ("cb3", C.c_long), ("aW3", C.c_long), ("ab3", C.c_long),
                ("bW3", C.c_long), ("bb3", C.c_long), ("ntensors", C.c_int),
                ("t_off", C.c_long * MAX_T), ("t_len", C.c_long * MAX_T), ("t_grad", C.c_int * MAX_T)]


MAX_CT, NCONV = 40, 6


class CarlaLayout(C.Structure):  # include/ppo_carla.h
    _fields_ = [("C", C.c_int), ("IH", C.c_int), ("IW", C.c_int), ("NM", C.c_int), ("NV", C.c_int), ("A", C.c_int),
                ("P", C.c_long), ("hi", C.c_long), ("lo", C.c_long),
                ("conv_w", C.c_long * NCONV), ("conv_b", C.c_long * NCONV),
                ("conv_ic", C.c_int * NCONV), ("conv_oc", C.c_int * NCONV), ("conv_k", C.c_int * NCONV),
                ("conv_s", C.c_int * NCONV), ("conv_ih", C.c_int * NCONV), ("conv_iw", C.c_int * NCONV),
                ("conv_oh", C.c_int * NCONV), ("conv_ow", C.c_int * NCONV),
                ("lin_w", C.c_long * 2), ("lin_b", C.c_long * 2), ("st_w", C.c_long * 2), ("st_b", C.c_long * 2),
                ("v_w", C.c_long * 3), ("v_b", C.c_long * 3), ("pi_w", C.c_long * 2), ("pi_b", C.c_long * 2),
                ("mu_w", C.c_long), ("mu_b", C.c_long), ("sg_w", C.c_long), ("sg_b", C.c_long),
                ("ntensors", C.c_int), ("t_off", C.c_long * MAX_CT), ("t_len", C.c_long * MAX_CT),
                ("t_grad", C.c_int * MAX_CT)]


class CarlaTrainConfig(C.Structure):  # ppo_carla_train_config; defaults = carla_config.h:31-40
    _fields_ = [("clip_coef", C.c_float), ("ent_coef", C.c_float), ("vf_coef", C.c_float),
                ("max_grad_norm", C.c_float), ("adam_eps", C.c_float), ("norm_adv", C.c_int), ("clip_vloss", C.c_int)]


class CarlaUpdateStats(C.Structure):
    _fields_ = [("pg_loss", C.c_float), ("v_loss", C.c_float), ("entropy", C.c_float),
                ("old_approx_kl", C.c_float), ("approx_kl", C.c_float), ("clipfrac", C.c_float),
                ("grad_norm", C.c_float)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class CarlaConfig(C.Structure):  # ppo_carla_config; defaults = carla_config.h
    _fields_ = [("obs_channels", C.c_int), ("bev_h", C.c_int), ("bev_w", C.c_int), ("num_measurements", C.c_int),
                ("num_value_measurements", C.c_int), ("action_dim", C.c_int), ("beta_min", C.c_float),
                ("max_batch", C.c_int), ("seed", C.c_uint64), ("rank", C.c_int)]


PPO_CARLA_SAMPLE, PPO_CARLA_MEAN, PPO_CARLA_GIVEN, PPO_CARLA_ROACH = range(4)

_LIB = None

# (name, restype, argtypes) of every entry point declared in include/ppo_hip.h / ppo_synth_env.h /
# ppo_carla.h / ppo_pth.h
_VP, _FP, _I, _L, _F, _SZ = C.c_void_p, C.c_void_p, C.c_int, C.c_long, C.c_float, C.c_size_t
SYMBOLS = [
    ("ppo_last_error", C.c_char_p, []),
    ("ppo_runtime_check", _I, []),
    ("ppo_version", C.c_char_p, []),
    ("ppo_obs_norm", _I, [C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.POINTER(C.c_float)),
                          C.POINTER(_I)]),
    ("ppo_create", _I, [C.POINTER(HipConfig), _I, C.POINTER(_VP)]),
    ("ppo_create_ex", _I, [C.POINTER(HipConfig), _I, C.c_char_p, C.POINTER(_VP)]),
    ("ppo_destroy", _I, [_VP]),
    ("ppo_get_layout", _I, [_VP, C.POINTER(Layout)]),
    ("ppo_stream", _VP, [_VP]),
    ("ppo_load_params", _I, [_VP, _FP, _L]),
    ("ppo_save_params", _I, [_VP, _FP, _L]),
    ("ppo_save_adam", _I, [_VP, _FP, _FP, _L, C.POINTER(_L)]),
    ("ppo_load_adam", _I, [_VP, _FP, _FP, _L, _L]),
    ("ppo_get_action_and_value", _I, [_VP, _I, _FP, _I, _FP, _L, _L, _FP, _FP, _FP, _FP, _VP]),
    ("ppo_get_value", _I, [_VP, _I, _FP, _FP, _VP]),
    ("ppo_rollout_act", _I, [_VP, _I, _I, _I, _FP, _FP, _FP, _VP]),
    ("ppo_rollout_values", _I, [_VP, _VP]),
    ("ppo_rollout_reward", _I, [_VP, _I, _I, _I, _FP, _VP]),
    ("ppo_compute_gae", _I, [_VP, _FP, _FP, _I, _VP]),
    ("ppo_gae_from_values", _I, [_VP, _FP, _FP, _I, _VP]),
    ("ppo_update", _I, [_VP, _F, _VP, C.POINTER(UpdateStats)]),
    ("ppo_update_ex", _I, [_VP, _F, _I, _VP, C.POINTER(UpdateStats)]),
    ("ppo_sync", _I, [_VP]),
    ("ppo_debug_last_grad", _I, [_VP, _FP, _L]),
    ("ppo_snapshot_state", _I, [_VP]),
    ("ppo_read_snapshot", _I, [_VP, _FP, _FP, _FP, _L, C.POINTER(_L)]),
    ("ppo_iteration", _L, [_VP]),
    ("ppo_set_iteration", _I, [_VP, _L]),
    ("ppo_buffer", _VP, [_VP, _I]),
    ("ppo_comm_unique_id", _I, [C.c_char_p]),
    ("ppo_comm_init", _I, [_VP, C.c_char_p, _I, _I]),
    ("ppo_comm_init_host", _I, [_VP, _I, _I, C.c_void_p, _VP]),
    ("ppo_comm_destroy", _I, [_VP]),
    ("ppo_comm_broadcast_params", _I, [_VP, _I]),
    ("ppo_comm_allreduce", _I, [_VP, _FP, _L, _I]),
    ("ppo_comm_info", _I, [_VP, C.POINTER(_I), C.POINTER(_I), C.POINTER(_I)]),
    ("ppo_get_device", _I, [_VP, C.POINTER(_I), C.c_char_p, _I]),
    ("ppo_kernel_info", _I, [_VP, C.c_char_p, _I]),
    ("ppo_set_device", _I, [_I]),
    ("ppo_device_count", _I, [C.POINTER(_I)]),
    ("ppo_dev_malloc", _I, [C.POINTER(_VP), _SZ]),
    ("ppo_dev_free", _I, [_VP]),
    ("ppo_memcpy_h2d", _I, [_VP, _VP, _SZ]),
    ("ppo_memcpy_d2h", _I, [_VP, _VP, _SZ]),
    ("ppo_memset_dev", _I, [_VP, _I, _SZ]),
    ("ppo_device_sync", _I, []),
    ("ppo_profile_enable", _I, [_VP, _I]),
    ("ppo_profile_read", _I, [_VP, C.POINTER(C.c_double), C.POINTER(_L), _I]),
    ("ppo_profile_name", C.c_char_p, [_I]),
    ("ppo_profile_reset", _I, [_VP]),
    ("psyn_create", _I, [_I, _I, _I, C.POINTER(_VP)]),
    ("psyn_destroy", _I, [_VP]),
    ("psyn_reset", _I, [_VP, _I, _FP, _FP, _VP]),
    ("psyn_step", _I, [_VP, _I, _I, _FP, _F, _F, _FP, _FP, _FP, _VP]),
    ("psyn_episode_stats", _I, [_VP, C.POINTER(_F), C.POINTER(_F), C.POINTER(_F)]),
    ("psyn_episode_stats_begin", _I, [_VP, _VP]),
    ("psyn_episode_stats_end", _I, [_VP, C.POINTER(_F), C.POINTER(_F), C.POINTER(_F)]),
    ("ppo_rollout_synth", _I, [_VP, _VP, _FP, _FP, _FP, _FP]),
    ("psyn_set_action_space", _I, [_VP, _F, _F]),
    ("ppo_set_rollout_mode", _I, [_VP, _I]),
    ("psyn_action_space", _I, [_VP, C.POINTER(_F), C.POINTER(_F)]),
    ("psyn_attach_wrappers", _I, [_VP, _VP]),
    ("pwrap_create", _I, [_I, _I, _F, C.POINTER(_VP)]),
    ("pwrap_destroy", _I, [_VP]),
    ("pwrap_reset", _I, [_VP, _I, _I, _FP, _VP]),
    ("pwrap_step", _I, [_VP, _I, _I, _FP, _FP, _FP, _FP, _VP]),
    ("pwrap_read_state", _I, [_VP, _FP, _L]),
    ("ppo_carla_create", _I, [C.POINTER(CarlaConfig), _I, C.POINTER(_VP)]),
    ("ppo_carla_create_ex", _I, [C.POINTER(CarlaConfig), _I, C.c_char_p, C.POINTER(_VP)]),
    ("ppo_carla_destroy", _I, [_VP]),
    ("ppo_carla_get_layout", _I, [_VP, C.POINTER(CarlaLayout)]),
    ("ppo_carla_load_params", _I, [_VP, _FP, _L]),
    ("ppo_carla_forward", _I, [_VP, _I, _VP, _FP, _FP, _I, _FP, _L, _L, _FP, _FP, _FP, _FP, _FP, _FP, _VP]),
    ("ppo_carla_update", _I, [_VP, C.POINTER(CarlaTrainConfig), _I, _VP, _FP, _FP, _FP, _FP, _FP, _FP, _FP, _F,
                              C.POINTER(CarlaUpdateStats), _VP]),
    ("ppo_carla_save_params", _I, [_VP, _FP, _L]),
    ("ppo_carla_last_grad", _I, [_VP, _FP, _L]),
    ("ppo_carla_save_adam", _I, [_VP, _FP, _FP, _L, C.POINTER(_L)]),
    ("ppo_carla_load_adam", _I, [_VP, _FP, _FP, _L, _L]),
    ("ppo_carla_comm_init", _I, [_VP, C.c_char_p, _I, _I]),
    ("ppo_carla_comm_broadcast_params", _I, [_VP, _I]),
    ("ppo_layout_fill", _I, [C.POINTER(Layout), _I, _I, _I, _I]),
    ("ppo_carla_layout_fill", _I, [C.POINTER(CarlaLayout), _I, _I, _I, _I, _I, _I]),
    ("ppo_pth_save_agent", _I, [C.POINTER(Layout), _FP, C.c_char_p]),
    ("ppo_pth_load_agent", _I, [C.POINTER(Layout), C.c_char_p, _FP, _L]),
    ("ppo_pth_save_adam", _I, [C.POINTER(Layout), _FP, _FP, _L, C.c_double, C.c_double, C.c_char_p]),
    ("ppo_pth_load_adam", _I, [C.POINTER(Layout), C.c_char_p, _FP, _FP, _L, C.POINTER(_L),
                               C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("ppo_carla_pth_save", _I, [C.POINTER(CarlaLayout), _FP, C.c_char_p]),
    ("ppo_carla_pth_load", _I, [C.POINTER(CarlaLayout), C.c_char_p, _FP, _L]),
]


def build_library(quiet=True):
    """Compiles libppo_hip.so in-tree (hipcc --offload-arch=gfx950)."""
    cmd = ["make", "-C", PKG_ROOT, "-j4"]
    subprocess.check_call(cmd, stdout=subprocess.DEVNULL if quiet else None)


def lib():
    """Loads libppo_hip.so. Raises if it is missing: there is no fallback path."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise PPOError(f"libppo_hip.so not built ({LIB_PATH}); run `make -C {PKG_ROOT}` or "
                           "__graft_entry__.build()")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, res, args in SYMBOLS:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = L
    return _LIB


def check(rc):
    if rc != 0:
        raise PPOError(f"libppo_hip error {rc}: {lib().ppo_last_error().decode()}")


# ------------------------------------------------------------------------------------------------
# LibTorch checkpoints (include/ppo_pth.h): model_*.pth / optimizer_*.pth as torch::save writes them
# ------------------------------------------------------------------------------------------------
def agent_layout(kind, O, A, H) -> Layout:
    L = Layout()
    check(lib().ppo_layout_fill(C.byref(L), kind, O, A, H))
    return L


def carla_layout(C_=15, IH=192, IW=192, NM=8, NV=3, A=2) -> CarlaLayout:
    L = CarlaLayout()
    check(lib().ppo_carla_layout_fill(C.byref(L), C_, IH, IW, NM, NV, A))
    return L


def _f32(a, n):
    a = np.ascontiguousarray(a, dtype=np.float32).reshape(-1)
    if a.size != n:
        raise PPOError(f"expected {n} floats, got {a.size}")
    return a


def save_agent_pth(layout: Layout, params, path):
    """torch::save(agent, path) of the flat parameters (named_parameters() order)."""
    p = _f32(params, layout.P)
    check(lib().ppo_pth_save_agent(C.byref(layout), p.ctypes.data, os.fsencode(path)))


def load_agent_pth(layout: Layout, path):
    """torch::load(agent, path) -> flat parameters."""
    out = np.empty(layout.P, np.float32)
    check(lib().ppo_pth_load_agent(C.byref(layout), os.fsencode(path), out.ctypes.data, layout.P))
    return out


def save_adam_pth(layout: Layout, m, v, step, lr, eps, path):
    """torch::save(optimizer, path) of an Adam(agent->parameters(), AdamOptions(lr).eps(eps))."""
    m, v = _f32(m, layout.P), _f32(v, layout.P)
    check(lib().ppo_pth_save_adam(C.byref(layout), m.ctypes.data, v.ctypes.data, int(step), float(lr), float(eps),
                                  os.fsencode(path)))


def load_adam_pth(layout: Layout, path):
    """torch::load(optimizer, path) -> (exp_avg, exp_avg_sq, step, lr, eps)."""
    m, v = np.empty(layout.P, np.float32), np.empty(layout.P, np.float32)
    step, lr, eps = C.c_long(0), C.c_double(0), C.c_double(0)
    check(lib().ppo_pth_load_adam(C.byref(layout), os.fsencode(path), m.ctypes.data, v.ctypes.data, layout.P,
                                  C.byref(step), C.byref(lr), C.byref(eps)))
    return m, v, step.value, lr.value, eps.value


def save_carla_pth(layout: CarlaLayout, params, path):
    p = _f32(params, layout.P)
    check(lib().ppo_carla_pth_save(C.byref(layout), p.ctypes.data, os.fsencode(path)))


def load_carla_pth(layout: CarlaLayout, path):
    out = np.empty(layout.P, np.float32)
    check(lib().ppo_carla_pth_load(C.byref(layout), os.fsencode(path), out.ctypes.data, layout.P))
    return out


def obs_norm(env_id):
    """(mean, std) the AC agent normalises observations with for env_id (ac:480-534); None for
    HalfCheetah-v5 (zeros / ones)."""
    m, s, n = C.POINTER(C.c_float)(), C.POINTER(C.c_float)(), C.c_int(0)
    check(lib().ppo_obs_norm(env_id.encode(), C.byref(m), C.byref(s), C.byref(n)))
    if n.value == 0:
        return None
    return (np.ctypeslib.as_array(m, shape=(n.value,)).copy(), np.ctypeslib.as_array(s, shape=(n.value,)).copy())


def device_count():
    n = C.c_int(0)
    check(lib().ppo_device_count(C.byref(n)))
    return n.value


def set_device(d):
    check(lib().ppo_set_device(d))


# ------------------------------------------------------------------------------------------------
# device memory
# ------------------------------------------------------------------------------------------------
class DeviceArray:
    """A float32 / int32 HIP allocation with numpy copies in and out."""

    def __init__(self, shape, dtype=np.float32):
        self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape)) * self.dtype.itemsize
        p = C.c_void_p()
        check(lib().ppo_dev_malloc(C.byref(p), self.nbytes))
        self.ptr = p.value
        self._owned = True

    @classmethod
    def from_numpy(cls, a, dtype=None):
        a = np.ascontiguousarray(a, dtype=dtype or a.dtype)
        d = cls(a.shape, a.dtype)
        d.upload(a)
        return d

    @classmethod
    def wrap(cls, ptr, shape, dtype=np.float32):
        d = cls.__new__(cls)
        d.shape = tuple(shape)
        d.dtype = np.dtype(dtype)
        d.nbytes = int(np.prod(d.shape)) * d.dtype.itemsize
        d.ptr = ptr
        d._owned = False
        return d

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        assert a.nbytes == self.nbytes, (a.nbytes, self.nbytes)
        check(lib().ppo_memcpy_h2d(self.ptr, a.ctypes.data, self.nbytes))

    def numpy(self):
        out = np.empty(self.shape, self.dtype)
        check(lib().ppo_memcpy_d2h(out.ctypes.data, self.ptr, self.nbytes))
        return out

    def zero(self):
        check(lib().ppo_memset_dev(self.ptr, 0, self.nbytes))

    def free(self):
        if self._owned and self.ptr:
            lib().ppo_dev_free(self.ptr)
        self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


# ------------------------------------------------------------------------------------------------
# configs (reference GlobalConfig names and defaults)
# ------------------------------------------------------------------------------------------------
ENV_DIMS = {  # obs / act dims and action bounds of the reference's MuJoCo envs
    "HalfCheetah-v5": (17, 6, -1.0, 1.0),   # libs/gymcpp/mujoco/half_cheetah_v5.h:31-34
    "Humanoid-v4": (376, 17, -0.4, 0.4),    # humanoid_v4.h:27-30
    "Ant-v5": (105, 8, -1.0, 1.0),          # ant_v5.h:38-41
    "Hopper-v5": (11, 3, -1.0, 1.0),        # hopper_v5.h:35-38
}


@dataclass
class PPOConfig:
    """GlobalConfig of ppo_continuous_action (src/ppo_continuous_action.cpp:51-118)."""
    seed: int = 1
    eval_seed: int = 2
    total_timesteps: int = 1_000_000
    learning_rate: float = 3e-4
    num_envs: int = 1
    num_steps: int = 2048
    gamma: float = 0.99
    gae_lambda: float = 0.95
    num_minibatches: int = 32
    update_epochs: int = 10
    norm_adv: bool = True
    clip_coef: float = 0.2
    clip_vloss: bool = True
    ent_coef: float = 0.0
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    adam_eps: float = 1e-5
    anneal_lr: bool = True
    num_eval_runs: int = 10
    clip_actions: bool = True
    torch_deterministic: bool = True
    exp_name_stem: str = "PPO_002"
    env_id: str = "Humanoid-v4"
    net_kind: int = PPO_NET_TANH_NORMAL
    hidden: int = 64

    @property
    def batch_size(self):
        return self.num_steps * self.num_envs

    @property
    def minibatch_size(self):
        return self.batch_size // self.num_minibatches

    @property
    def num_iterations(self):
        return self.total_timesteps // self.batch_size


@dataclass
class ACPPOConfig(PPOConfig):
    """GlobalConfig of ac_ppo_continuous_action (src/ac_ppo_continuous_action.cpp:55-148)."""
    total_timesteps: int = 10_000_000
    learning_rate: float = 2.5e-4
    num_envs: int = 8
    num_steps: int = 128
    num_minibatches: int = 4
    update_epochs: int = 4
    clip_coef: float = 0.1
    ent_coef: float = 0.01
    num_eval_runs: int = 128
    exp_name_stem: str = "Ant-v5_AC_PPO_Atari"
    env_id: str = "Ant-v5"
    gpu_ids: list = field(default_factory=lambda: [0])
    collect_device: str = "cpu"
    train_device: str = "cpu"
    use_dd_ppo_preempt: int = 0
    net_kind: int = PPO_NET_LN_BETA
    hidden: int = 256


def hip_config(cfg: PPOConfig, num_envs_per_device=None, rank=0, world_size=1) -> HipConfig:
    O, A, _, _ = ENV_DIMS[cfg.env_id] if cfg.env_id in ENV_DIMS else (cfg.obs_dim, cfg.act_dim, -1, 1)
    E = num_envs_per_device if num_envs_per_device is not None else cfg.num_envs
    return HipConfig(cfg.net_kind, O, A, cfg.hidden, E, cfg.num_steps, cfg.num_minibatches, cfg.update_epochs,
                     cfg.gamma, cfg.gae_lambda, cfg.clip_coef, cfg.ent_coef, cfg.vf_coef, cfg.max_grad_norm,
                     cfg.adam_eps, int(cfg.norm_adv), int(cfg.clip_vloss), cfg.seed, rank, world_size)


# ------------------------------------------------------------------------------------------------
# agent / trainer context
# ------------------------------------------------------------------------------------------------
class Agent:
    """Owns a ppo_t: the agent parameters, the Adam state and the [T, E, *] rollout storage."""

    def __init__(self, hcfg: HipConfig, device=0, options: str | None = None):
        """options: ppo_create_ex kernel selection, e.g. "upd_kernel=fwdbwd,dw_fused=0" (A/B tests)."""
        self.hcfg = hcfg
        h = C.c_void_p()
        check(lib().ppo_create_ex(C.byref(hcfg), device, options.encode() if options else None, C.byref(h)))
        self.h = h.value
        self.layout = Layout()
        check(lib().ppo_get_layout(self.h, C.byref(self.layout)))
        self.num_params = self.layout.P
        self.O, self.A = hcfg.obs_dim, hcfg.act_dim

    def close(self):
        if getattr(self, "h", None):
            lib().ppo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- parameters ------------------------------------------------------------------------
    def load_params(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        check(lib().ppo_load_params(self.h, flat.ctypes.data, flat.size))

    def params(self):
        out = np.zeros(self.num_params, np.float32)
        check(lib().ppo_save_params(self.h, out.ctypes.data, out.size))
        return out

    def adam_state(self):
        m = np.zeros(self.num_params, np.float32)
        v = np.zeros(self.num_params, np.float32)
        st = C.c_long()
        check(lib().ppo_save_adam(self.h, m.ctypes.data, v.ctypes.data, m.size, C.byref(st)))
        return m, v, st.value

    def load_adam(self, m, v, step):
        """Set the Adam moments (flat, unpadded named_parameters() order) and the step count."""
        m, v = np.ascontiguousarray(m, np.float32), np.ascontiguousarray(v, np.float32)
        check(lib().ppo_load_adam(self.h, m.ctypes.data, v.ctypes.data, m.size, int(step)))

    # -- agent calls (device arrays in / out) ----------------------------------------------------
    def get_action_and_value(self, x: DeviceArray, sample_type=PPO_SAMPLE, action: DeviceArray | None = None,
                             env_base=0, step_id=0):
        n = x.shape[0]
        act = DeviceArray((n, self.A)); lp = DeviceArray(n); ent = DeviceArray(n); val = DeviceArray(n)
        check(lib().ppo_get_action_and_value(self.h, n, x.ptr, sample_type, action.ptr if action else None,
                                             env_base, step_id, act.ptr, lp.ptr, ent.ptr, val.ptr, None))
        return act, lp, ent, val

    def get_value(self, x: DeviceArray):
        n = x.shape[0]
        val = DeviceArray(n)
        check(lib().ppo_get_value(self.h, n, x.ptr, val.ptr, None))
        return val

    def buffer(self, which, shape):
        return DeviceArray.wrap(lib().ppo_buffer(self.h, which), shape)

    def rollout_act(self, step, e0, e1, next_obs: DeviceArray, next_done: DeviceArray, action_out=None):
        check(lib().ppo_rollout_act(self.h, step, e0, e1, next_obs.ptr, next_done.ptr,
                                    action_out.ptr if action_out else None, None))

    def rollout_values(self):
        """The deferred critic pass of rollout_act (values of every step acted since the last pass)."""
        check(lib().ppo_rollout_values(self.h, None))

    def rollout_reward(self, step, e0, e1, reward: DeviceArray):
        check(lib().ppo_rollout_reward(self.h, step, e0, e1, reward.ptr, None))

    def compute_gae(self, next_obs: DeviceArray, next_done: DeviceArray, nsteps=None):
        check(lib().ppo_compute_gae(self.h, next_obs.ptr, next_done.ptr, nsteps or self.hcfg.num_steps, None))

    def gae_from_values(self, next_value: DeviceArray, next_done: DeviceArray, nsteps=None):
        check(lib().ppo_gae_from_values(self.h, next_value.ptr, next_done.ptr, nsteps or self.hcfg.num_steps, None))

    def update(self, lr, perms: DeviceArray | None = None, want_stats=True, num_steps_collected=None):
        """num_steps_collected < num_steps: a DD-PPO partial collection (ppo_update_ex)."""
        st = UpdateStats()
        check(lib().ppo_update_ex(self.h, lr, num_steps_collected or self.hcfg.num_steps, perms.ptr if perms else None,
                                  C.byref(st) if want_stats else None))
        return st.as_dict() if want_stats else None

    def sync(self):
        check(lib().ppo_sync(self.h))

    def last_grad(self):
        out = np.zeros(self.num_params, np.float32)
        check(lib().ppo_debug_last_grad(self.h, out.ctypes.data, out.size))
        return out

    @property
    def iteration(self):
        return lib().ppo_iteration(self.h)

    def set_iteration(self, it):
        check(lib().ppo_set_iteration(self.h, it))

    # -- profiling --------------------------------------------------------------------------------
    def profile(self, mask=0xFFFF):
        check(lib().ppo_profile_enable(self.h, mask))

    def profile_read(self):
        ms = (C.c_double * 32)()
        cnt = (C.c_long * 32)()
        n = lib().ppo_profile_read(self.h, ms, cnt, 32)
        return {lib().ppo_profile_name(i).decode(): (ms[i], cnt[i]) for i in range(n) if cnt[i] > 0}

    def profile_reset(self):
        check(lib().ppo_profile_reset(self.h))

    # -- data parallel (RCCL) ---------------------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib().ppo_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, uid: bytes, rank, world):
        check(lib().ppo_comm_init(self.h, uid, rank, world))

    def comm_init_host(self, rank, world, allreduce):
        """Attach the host-transport communicator: allreduce(np.ndarray float32, average: bool)
        reduces the array in place over all ranks (e.g. torch.distributed gloo, or MPI)."""
        def _cb(buf, n, average, _user):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(n,)), bool(average))
                return 0
            except Exception:  # noqa: BLE001 — reported to the library as a failed collective
                return 1
        self._host_cb = HOST_ALLREDUCE_FN(_cb)  # keep the trampoline alive while attached
        check(lib().ppo_comm_init_host(self.h, rank, world, C.cast(self._host_cb, C.c_void_p), None))

    def comm_destroy(self):
        check(lib().ppo_comm_destroy(self.h))
        self._host_cb = None

    def comm_broadcast_params(self, root=0):
        check(lib().ppo_comm_broadcast_params(self.h, root))

    def comm_allreduce(self, buf: DeviceArray, average=True):
        check(lib().ppo_comm_allreduce(self.h, buf.ptr, int(np.prod(buf.shape)), int(average)))
        self.sync()

    def device(self):
        """(device ordinal, PCI bus id) the context runs on (ppo_get_device)."""
        d = C.c_int(-1)
        bus = C.create_string_buffer(64)
        check(lib().ppo_get_device(self.h, C.byref(d), bus, 64))
        return d.value, bus.value.decode()

    def kernel_info(self):
        """The update / dW kernels this context selected (ppo_kernel_info)."""
        buf = C.create_string_buffer(256)
        check(lib().ppo_kernel_info(self.h, buf, 256))
        return buf.value.decode()

    def set_rollout_mode(self, per_step: bool):
        """ppo_rollout_synth: one persistent launch (default, where supported) or per-step launches."""
        check(lib().ppo_set_rollout_mode(self.h, 1 if per_step else 0))

    def comm_info(self):
        """(kind, rank, world) of the attached communicator: kind "none" / "rccl" / "host"; for RCCL
        rank and world are what the communicator itself reports (ncclCommUserRank / ncclCommCount)."""
        k, r, w = C.c_int(), C.c_int(), C.c_int()
        check(lib().ppo_comm_info(self.h, C.byref(k), C.byref(r), C.byref(w)))
        return ({0: "none", 1: "rccl", 2: "host"}[k.value], r.value, w.value)


class CarlaAgent:
    """The CaRL CNN agent (include/carla/carla_model.h AgentImpl) on the device.
    forward() mirrors AgentImpl::forward: returns (actions, log_prob, entropy, values, alpha, beta)
    as DeviceArrays; sample_type is "sample", "mean", "roach" or a given `actions` array."""

    _MODES = {"sample": PPO_CARLA_SAMPLE, "mean": PPO_CARLA_MEAN, "roach": PPO_CARLA_ROACH}

    def __init__(self, max_batch, obs_channels=15, bev=192, num_measurements=8, num_value_measurements=3,
                 action_dim=2, beta_min=1.0, seed=1, rank=0, device=0, options: str | None = None):
        self.cfg = CarlaConfig(obs_channels, bev, bev, num_measurements, num_value_measurements, action_dim, beta_min,
                               max_batch, seed, rank)
        self._h = C.c_void_p()
        check(lib().ppo_carla_create_ex(C.byref(self.cfg), device, options.encode() if options else None,
                                        C.byref(self._h)))
        self.layout = CarlaLayout()
        check(lib().ppo_carla_get_layout(self._h, C.byref(self.layout)))

    def close(self):
        if self._h:
            lib().ppo_carla_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def load_params(self, flat):
        flat = np.ascontiguousarray(flat, np.float32)
        check(lib().ppo_carla_load_params(self._h, flat.ctypes.data_as(C.c_void_p), flat.size))

    def forward(self, bev: DeviceArray, meas: DeviceArray, vmeas: DeviceArray, actions: DeviceArray | None = None,
                sample_type="sample", env_base=0, step_id=0, out=None, sync=True):
        """(action, logprob, entropy, value, alpha, beta); out: preallocated arrays of those shapes."""
        n, A = bev.shape[0], self.layout.A
        mode = PPO_CARLA_GIVEN if actions is not None else self._MODES[sample_type]
        if out is None:
            out = [DeviceArray((n, A)), DeviceArray((n,)), DeviceArray((n,)), DeviceArray((n,)), DeviceArray((n, A)),
                   DeviceArray((n, A))]
        check(lib().ppo_carla_forward(self._h, n, bev.ptr, meas.ptr, vmeas.ptr, mode,
                                      actions.ptr if actions is not None else None, env_base, step_id,
                                      *[o.ptr for o in out], None))
        if sync:
            check(lib().ppo_device_sync())
        return tuple(out)

    def update(self, bev: DeviceArray, meas: DeviceArray, vmeas: DeviceArray, actions: DeviceArray,
               old_logp: DeviceArray, adv: DeviceArray, ret: DeviceArray, old_v: DeviceArray, lr=3e-4,
               clip_coef=0.2, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, adam_eps=1e-5, norm_adv=True,
               clip_vloss=True, want_stats=True):
        """One minibatch of ac_ppo_carla.cpp:540-619 (loss, backward, clip_grad_norm_, Adam)."""
        tc = CarlaTrainConfig(clip_coef, ent_coef, vf_coef, max_grad_norm, adam_eps, int(norm_adv), int(clip_vloss))
        st = CarlaUpdateStats()
        check(lib().ppo_carla_update(self._h, C.byref(tc), bev.shape[0], bev.ptr, meas.ptr, vmeas.ptr, actions.ptr,
                                     old_logp.ptr, adv.ptr, ret.ptr, old_v.ptr, lr,
                                     C.byref(st) if want_stats else None, None))
        return st.as_dict() if want_stats else None

    def params(self):
        out = np.empty(self.layout.P, np.float32)
        check(lib().ppo_carla_save_params(self._h, out.ctypes.data, out.size))
        return out

    def last_grad(self):
        out = np.empty(self.layout.P, np.float32)
        check(lib().ppo_carla_last_grad(self._h, out.ctypes.data, out.size))
        return out

    def adam_state(self):
        m, v, step = np.empty(self.layout.P, np.float32), np.empty(self.layout.P, np.float32), C.c_long(0)
        check(lib().ppo_carla_save_adam(self._h, m.ctypes.data, v.ctypes.data, m.size, C.byref(step)))
        return m, v, step.value

    def load_adam(self, m, v, step):
        m, v = np.ascontiguousarray(m, np.float32), np.ascontiguousarray(v, np.float32)
        check(lib().ppo_carla_load_adam(self._h, m.ctypes.data, v.ctypes.data, m.size, int(step)))

    def comm_init(self, uid: bytes, rank=0, world=1):
        """Attach an RCCL communicator (ac_ppo_carla.cpp:561-616 data parallelism); uid from
        Agent.comm_unique_id()."""
        check(lib().ppo_carla_comm_init(self._h, uid, rank, world))

    def comm_broadcast_params(self, root=0):
        check(lib().ppo_carla_comm_broadcast_params(self._h, root))


class SynthEnv:
    """Device-resident synthetic HalfCheetah-shaped vector env (include/ppo_synth_env.h)."""

    def __init__(self, num_envs, obs_dim, act_dim):
        h = C.c_void_p()
        check(lib().psyn_create(num_envs, obs_dim, act_dim, C.byref(h)))
        self.h = h.value
        self.E, self.O, self.A = num_envs, obs_dim, act_dim

    def reset(self, seed, obs: DeviceArray, done: DeviceArray, stream=None):
        check(lib().psyn_reset(self.h, seed, obs.ptr, done.ptr, stream))

    def step(self, action: DeviceArray, obs: DeviceArray, reward: DeviceArray, done: DeviceArray, lo=-1.0, hi=1.0,
             e0=0, e1=None, stream=None):
        check(lib().psyn_step(self.h, e0, e1 if e1 is not None else self.E, action.ptr, lo, hi, obs.ptr, reward.ptr,
                              done.ptr, stream))

    def episode_stats(self):
        r, l_, n = C.c_float(), C.c_float(), C.c_float()
        check(lib().psyn_episode_stats(self.h, C.byref(r), C.byref(l_), C.byref(n)))
        return r.value, l_.value, n.value

    def set_action_space(self, lo, hi):
        check(lib().psyn_set_action_space(self.h, lo, hi))

    def attach_wrappers(self, wrappers: "EnvWrappers | None"):
        """Run the wrapper chain inside the env's own kernels (psyn_attach_wrappers); None detaches."""
        check(lib().psyn_attach_wrappers(self.h, wrappers.h if wrappers is not None else None))
        self._wrappers = wrappers  # keep the state alive while attached

    def close(self):
        if getattr(self, "h", None):
            lib().psyn_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EnvWrappers:
    """The PPO trainer's env wrapper chain on the device (include/ppo_env_wrappers.h; ppo:41-49):
    NormalizeObservation -> clamp -> NormalizeReward -> clamp, one state per env in HBM."""

    def __init__(self, num_envs, obs_dim, gamma=0.99):
        h = C.c_void_p()
        check(lib().pwrap_create(num_envs, obs_dim, gamma, C.byref(h)))
        self.h = h.value
        self.E, self.O, self.gamma = num_envs, obs_dim, gamma

    def reset(self, obs: DeviceArray, e0=0, e1=None, stream=None):
        check(lib().pwrap_reset(self.h, e0, self.E if e1 is None else e1, obs.ptr, stream))

    def step(self, obs: DeviceArray, reward: DeviceArray, term: DeviceArray | None = None,
             is_reset: DeviceArray | None = None, e0=0, e1=None, stream=None):
        check(lib().pwrap_step(self.h, e0, self.E if e1 is None else e1, obs.ptr, reward.ptr,
                               term.ptr if term is not None else None, is_reset.ptr if is_reset is not None else None,
                               stream))

    def state(self):
        """dict of the per-env state: obs_mean / obs_var [E,O], obs_count, rew_mean, rew_var, rew_acc,
        rew_count [E]"""
        E, O = self.E, self.O
        h = np.empty(2 * E * O + 5 * E, np.float32)
        check(lib().pwrap_read_state(self.h, h.ctypes.data, h.size))
        t = h[2 * E * O:].reshape(5, E)
        return {"obs_mean": h[:E * O].reshape(E, O), "obs_var": h[E * O:2 * E * O].reshape(E, O), "obs_count": t[0],
                "rew_mean": t[1], "rew_var": t[2], "rew_acc": t[3], "rew_count": t[4]}

    def close(self):
        if getattr(self, "h", None):
            lib().pwrap_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Trainer:
    """The reference main() loop (ppo:375-586 / ac:624-950) on the device-resident synthetic env:
    lr anneal -> rollout (T x act + env step) -> GAE -> update. One call = one iteration."""

    def __init__(self, cfg: PPOConfig, num_envs_per_device=None, rank=0, world_size=1, device=0, params=None,
                 wrappers=None, options=None):
        """wrappers: the PPO env wrapper chain (ppo:41-49) on the device env; default = what the
        reference trainer uses: on for the PPO agent (ppo_continuous_action), off for the AC agent
        (ac_ppo_continuous_action wraps its envs in RecordEpisodeStatistics only, ac:50-53)."""
        self.cfg = cfg
        self.hcfg = hip_config(cfg, num_envs_per_device, rank, world_size)
        self.agent = Agent(self.hcfg, device, options=options)
        if params is None:
            params = init_params(self.agent.layout, seed=cfg.seed, env_id=cfg.env_id)
        self.agent.load_params(params)
        E, O, A = self.hcfg.num_envs, self.hcfg.obs_dim, self.hcfg.act_dim
        self.env = SynthEnv(E, O, A)
        if cfg.env_id in ENV_DIMS:
            self.env.set_action_space(ENV_DIMS[cfg.env_id][2], ENV_DIMS[cfg.env_id][3])
        if wrappers is None:
            wrappers = self.hcfg.net_kind == PPO_NET_TANH_NORMAL
        self.wrappers = EnvWrappers(E, O, cfg.gamma) if wrappers else None
        if self.wrappers is not None:
            self.env.attach_wrappers(self.wrappers)
        self.next_obs = DeviceArray((E, O))
        self.next_done = DeviceArray(E)
        self.act_scratch = DeviceArray((E, A))
        self.rew_scratch = DeviceArray(E)
        self.env.reset(cfg.seed, self.next_obs, self.next_done, lib().ppo_stream(self.agent.h))
        self.num_iterations = max(1, cfg.num_iterations)
        self.iteration = 0
        self.global_step = 0
        self.last_stats = None

    def lr_now(self):
        if not self.cfg.anneal_lr:
            return self.cfg.learning_rate
        frac = np.float32(1.0) - np.float32(self.iteration) / np.float32(self.num_iterations)
        return float(np.float32(frac * np.float32(self.cfg.learning_rate)))

    def rollout(self):
        check(lib().ppo_rollout_synth(self.agent.h, self.env.h, self.next_obs.ptr, self.next_done.ptr,
                                      self.act_scratch.ptr, self.rew_scratch.ptr))

    def iterate(self, want_stats=False):
        lr = self.lr_now()
        self.rollout()
        self.agent.compute_gae(self.next_obs, self.next_done)
        st = self.agent.update(lr, want_stats=want_stats)
        self.iteration += 1
        self.global_step += self.hcfg.num_envs * self.hcfg.num_steps * self.hcfg.world_size
        self.last_stats = st
        return st

    def close(self):
        self.agent.close()
        self.env.close()
        if self.wrappers is not None:
            self.wrappers.close()


def init_params(layout: Layout, seed=1, env_id=None, obs_mean=None, obs_std=None):
    """Deterministic initial parameters in the reference's flat order.

    The reference initialises with LibTorch's RNG (orthogonal_ for the PPO agent, ppo:159-164; the
    nn::Linear / LayerNorm defaults for the AC agent, ac:159-186) which cannot be reproduced
    outside LibTorch; runs that need the reference's exact initial weights load them with
    Agent.load_params. This initialiser follows the same scales: orthogonal rows (gain sqrt(2),
    1.0 for the critic output, 0.01 for the actor output) for the PPO agent, kaiming-uniform
    (bound 1/sqrt(fan_in)) Linear weights and LayerNorm gamma=1, beta=0 for the AC agent."""
    rng = np.random.default_rng(seed)
    P = np.zeros(layout.P, np.float32)
    L = layout
    H, O, A = L.H, L.O, L.A

    def orth(rows, cols, gain):
        a = rng.standard_normal((max(rows, cols), min(rows, cols)))
        q, r = np.linalg.qr(a)
        q = q * np.sign(np.diag(r))
        q = q if rows >= cols else q.T
        return (gain * q[:rows, :cols]).astype(np.float32)

    def put(off, arr):
        P[off:off + arr.size] = arr.reshape(-1)

    def unif(rows, cols):
        b = 1.0 / np.sqrt(cols)
        return rng.uniform(-b, b, (rows, cols)).astype(np.float32)

    if L.kind == PPO_NET_TANH_NORMAL:
        g2 = np.sqrt(2.0)
        for tr, outW, outb, n_out, gain in ((L.critic, L.cW3, L.cb3, 1, 1.0), (L.actor, L.aW3, L.ab3, A, 0.01)):
            put(tr[0], orth(H, O, g2)); put(tr[4], orth(H, H, g2))
            put(outW, orth(n_out, H, gain))
        put(L.logstd, np.zeros(A, np.float32))
    else:
        lo, hi = -1.0, 1.0
        if env_id in ENV_DIMS:
            lo, hi = ENV_DIMS[env_id][2], ENV_DIMS[env_id][3]
        P[L.hi] = hi
        P[L.lo] = lo
        if obs_mean is None and env_id in ENV_DIMS and ENV_DIMS[env_id][0] == O:
            table = obs_norm(env_id)
            if table is not None:
                obs_mean, obs_std = table
        put(L.omean, np.zeros(O, np.float32) if obs_mean is None else np.asarray(obs_mean, np.float32))
        put(L.ostd, np.ones(O, np.float32) if obs_std is None else np.asarray(obs_std, np.float32))
        for tr in (L.critic, L.actor):
            put(tr[0], unif(H, O)); put(tr[1], rng.uniform(-1 / np.sqrt(O), 1 / np.sqrt(O), H).astype(np.float32))
            put(tr[2], np.ones(H, np.float32)); put(tr[3], np.zeros(H, np.float32))
            put(tr[4], unif(H, H)); put(tr[5], rng.uniform(-1 / 16, 1 / 16, H).astype(np.float32))
            put(tr[6], np.ones(H, np.float32)); put(tr[7], np.zeros(H, np.float32))
        put(L.cW3, unif(1, H)); P[L.cb3] = rng.uniform(-1 / 16, 1 / 16)
        put(L.aW3, unif(A, H)); put(L.ab3, rng.uniform(-1 / 16, 1 / 16, A).astype(np.float32))
        put(L.bW3, unif(A, H)); put(L.bb3, rng.uniform(-1 / 16, 1 / 16, A).astype(np.float32))
    return P
