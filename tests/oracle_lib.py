"""ctypes binding of oracle/liboracle.so — the CPU checker (test infrastructure only)."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

MAX_T = 32


class Layout(C.Structure):
    _fields_ = [("kind", C.c_int), ("O", C.c_int), ("A", C.c_int), ("H", C.c_int),
                ("P", C.c_long), ("train_begin", C.c_long),
                ("hi", C.c_long), ("lo", C.c_long), ("omean", C.c_long), ("ostd", C.c_long),
                ("logstd", C.c_long),
                ("critic", C.c_long * 8), ("actor", C.c_long * 8),
                ("cW3", C.c_long), ("cb3", C.c_long), ("aW3", C.c_long), ("ab3", C.c_long),
                ("bW3", C.c_long), ("bb3", C.c_long),
                ("ntensors", C.c_int),
                ("t_off", C.c_long * MAX_T), ("t_len", C.c_long * MAX_T), ("t_grad", C.c_int * MAX_T)]


class LossCfg(C.Structure):
    _fields_ = [("clip_coef", C.c_float), ("ent_coef", C.c_float), ("vf_coef", C.c_float),
                ("clip_vloss", C.c_int), ("norm_adv", C.c_int)]


class EnvState(C.Structure):
    _fields_ = [("E", C.c_int), ("O", C.c_int), ("A", C.c_int),
                ("q", C.c_void_p), ("t", C.c_void_p), ("autoreset", C.c_void_p),
                ("rseed", C.c_void_p), ("rcount", C.c_void_p), ("ep_ret", C.c_void_p), ("ep_len", C.c_void_p)]


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ORACLE_DIR, "liboracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "liboracle.so"], cwd=ORACLE_DIR)
        _LIB = C.CDLL(path)
        _LIB.orc_digamma.restype = C.c_double
        _LIB.orc_digamma.argtypes = [C.c_double]
        _LIB.orc_trigamma.argtypes = [C.c_double]
        _LIB.orc_trigamma.restype = C.c_double
        _LIB.orc_clip_grad_norm.restype = C.c_double
        _LIB.orc_u01.restype = C.c_float
        _LIB.orc_mix32.restype = C.c_uint32
        _LIB.orc_perm_index.restype = C.c_long
    return _LIB


def fp(a):
    return a.ctypes.data_as(C.c_void_p)


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def layout_init(kind, O, A, H):
    """Python restatement of include/ppo_layout.h's ppo_layout_init (kept in sync by tests)."""
    L = Layout()
    cur = [0]
    tens = []

    def add(n, grad=1):
        off = cur[0]
        tens.append((off, n, grad))
        cur[0] += n
        return off

    L.kind, L.O, L.A, L.H = kind, O, A, H
    L.hi = L.lo = L.omean = L.ostd = L.logstd = L.bW3 = L.bb3 = -1
    if kind == 0:
        L.logstd = add(A)
        L.train_begin = 0
        c = [add(H * O), add(H), -1, -1, add(H * H), add(H), -1, -1]
        L.critic[:] = c
        L.cW3 = add(H); L.cb3 = add(1)
        a = [add(H * O), add(H), -1, -1, add(H * H), add(H), -1, -1]
        L.actor[:] = a
        L.aW3 = add(A * H); L.ab3 = add(A)
    else:
        L.hi = add(1, 0); L.lo = add(1, 0); L.omean = add(O, 0); L.ostd = add(O, 0)
        L.train_begin = cur[0]
        for k in range(2):
            t = [add(H * O), add(H), add(H), add(H), add(H * H), add(H), add(H), add(H)]
            if k == 0:
                L.critic[:] = t
                L.cW3 = add(H); L.cb3 = add(1)
            else:
                L.actor[:] = t
        L.aW3 = add(A * H); L.ab3 = add(A); L.bW3 = add(A * H); L.bb3 = add(A)
    L.P = cur[0]
    L.ntensors = len(tens)
    for i, (o, n, g) in enumerate(tens):
        L.t_off[i] = o; L.t_len[i] = n; L.t_grad[i] = g
    return L


def get_action_and_value(L, params, x, mode, action=None, seed=1, rank=0, env_base=0, step_id=0):
    x = f32(x); params = f32(params)
    n = x.shape[0]
    act = np.zeros((n, L.A), np.float32)
    lp = np.zeros(n, np.float32); ent = np.zeros(n, np.float32); v = np.zeros(n, np.float32)
    ain = f32(action) if action is not None else np.zeros((n, L.A), np.float32)
    lib().orc_get_action_and_value(C.byref(L), fp(params), C.c_int(n), fp(x), C.c_int(mode), fp(ain),
                                   C.c_uint64(seed), C.c_int(rank), C.c_long(env_base), C.c_long(step_id),
                                   fp(act), fp(lp), fp(ent), fp(v))
    return act, lp, ent, v


def adv_stats(adv):
    adv = f32(adv)
    m = C.c_float(); s = C.c_float()
    lib().orc_adv_stats(C.c_int(adv.size), fp(adv), C.byref(m), C.byref(s))
    return m.value, s.value


def minibatch_grad(L, params, x, action, old_logp, adv, ret, old_v, cfg, adv_mean=None, adv_std=None):
    M = x.shape[0]
    if adv_mean is None:
        adv_mean, adv_std = adv_stats(adv)
    grad = np.zeros(L.P, np.float32); stats = np.zeros(7, np.float32)
    args = [f32(a) for a in (params, x, action, old_logp, adv, ret, old_v)]
    lib().orc_minibatch_grad(C.byref(L), fp(args[0]), C.c_int(M), *[fp(a) for a in args[1:]],
                             C.c_float(adv_mean), C.c_float(adv_std), C.byref(cfg), fp(grad), fp(stats))
    return grad, stats


def minibatch_grad_parallel(L, params, x, action, old_logp, adv, ret, old_v, cfg, adv_mean=None, adv_std=None,
                            threads=None, chunk=4096):
    """minibatch_grad over large M: fixed row chunks on a thread pool (ctypes drops the GIL), partials
    added in chunk order in double, then finished exactly as the serial form. Equal to
    minibatch_grad up to the double-precision order of the row sums."""
    from concurrent.futures import ThreadPoolExecutor
    M = x.shape[0]
    if adv_mean is None:
        adv_mean, adv_std = adv_stats(adv)
    args = [f32(a) for a in (params, x, action, old_logp, adv, ret, old_v)]
    bounds = [(r, min(M, r + chunk)) for r in range(0, M, chunk)]
    threads = threads or max(1, min(len(bounds), int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1))

    def run(b):
        G = np.zeros(L.P, np.float64); s = np.zeros(6, np.float64)
        lib().orc_minibatch_grad_part(C.byref(L), fp(args[0]), C.c_int(M), C.c_int(b[0]), C.c_int(b[1]),
                                      *[fp(a) for a in args[1:]], C.c_float(adv_mean), C.c_float(adv_std),
                                      C.byref(cfg), fp(G), fp(s))
        return G, s

    with ThreadPoolExecutor(threads) as ex:
        parts = list(ex.map(run, bounds))
    G = np.zeros(L.P, np.float64); s = np.zeros(6, np.float64)
    for g, ss in parts:
        G += g; s += ss
    grad = np.zeros(L.P, np.float32); stats = np.zeros(7, np.float32)
    lib().orc_minibatch_finish(C.byref(L), C.c_int(M), fp(G), fp(s), C.byref(cfg), fp(grad), fp(stats))
    return grad, stats


def clip_grad_norm(L, grad, max_norm):
    g = f32(grad).copy()
    tn = lib().orc_clip_grad_norm(C.byref(L), fp(g), C.c_float(max_norm))
    return g, tn


def adam_step(L, params, grad, m, v, step, lr, eps):
    p = f32(params).copy(); m = f32(m).copy(); v = f32(v).copy()
    lib().orc_adam_step(C.byref(L), fp(p), fp(f32(grad)), fp(m), fp(v), C.c_long(step), C.c_float(lr), C.c_float(eps))
    return p, m, v


def gae(rewards, values, dones, next_value, next_done, gamma, lam):
    T, E = rewards.shape
    adv = np.zeros((T, E), np.float32); ret = np.zeros((T, E), np.float32)
    a = [f32(x) for x in (rewards, values, dones, next_value, next_done)]
    lib().orc_gae(C.c_int(T), C.c_int(E), *[fp(x) for x in a], C.c_float(gamma), C.c_float(lam), fp(adv), fp(ret))
    return adv, ret


def perm(B, seed, rank, epoch_counter):
    out = np.zeros(B, np.int64)
    lib().orc_perm(C.c_long(B), C.c_uint64(seed), C.c_int(rank), C.c_long(epoch_counter), fp(out))
    return out


def update(L, params, m, v, step, b_obs, b_act, b_logp, b_adv, b_ret, b_val, epochs, minibatches, lr,
           max_grad_norm, adam_eps, cfg, seed=1, rank=0, epoch_counter0=0, perms=None):
    p = f32(params).copy(); m = f32(m).copy(); v = f32(v).copy()
    st = C.c_long(step)
    stats = np.zeros(7, np.float32)
    arrs = [f32(a) for a in (b_obs, b_act, b_logp, b_adv, b_ret, b_val)]
    pp = fp(np.ascontiguousarray(perms, np.int64)) if perms is not None else None
    lib().orc_update(C.byref(L), fp(p), fp(m), fp(v), C.byref(st), C.c_long(b_logp.shape[0]), C.c_int(L.O),
                     C.c_int(L.A), *[fp(a) for a in arrs], C.c_int(epochs), C.c_int(minibatches), C.c_float(lr),
                     C.c_float(max_grad_norm), C.c_float(adam_eps), C.byref(cfg), C.c_uint64(seed), C.c_int(rank),
                     C.c_long(epoch_counter0), pp, fp(stats))
    return p, m, v, st.value, stats


class VecWrappers:
    """Oracle PPO wrapper chain behind a vector env (ppo:41-49; orc_vwrap_*), one state per env."""

    def __init__(self, E, O, gamma=0.99):
        self.E, self.O, self.gamma = E, O, gamma
        self.st = np.zeros(2 * E * O + 5 * E, np.float32)
        lib().orc_vwrap_init(fp(self.st), C.c_int(E), C.c_int(O))

    def reset(self, obs):
        obs = f32(obs).copy()
        lib().orc_vwrap_reset(fp(self.st), C.c_int(self.E), C.c_int(self.O), fp(obs))
        return obs

    def step(self, obs, reward, term, is_reset):
        obs = f32(obs).copy(); reward = f32(reward).copy()
        lib().orc_vwrap_step(fp(self.st), C.c_int(self.E), C.c_int(self.O), C.c_float(self.gamma), fp(obs), fp(reward),
                             fp(f32(term)), fp(f32(is_reset)))
        return obs, reward

    def state(self):
        E, O = self.E, self.O
        t = self.st[2 * E * O:].reshape(5, E)
        return {"obs_mean": self.st[:E * O].reshape(E, O), "obs_var": self.st[E * O:2 * E * O].reshape(E, O),
                "obs_count": t[0], "rew_mean": t[1], "rew_var": t[2], "rew_acc": t[3], "rew_count": t[4]}


def wrappers_script(O, T, reset_at):
    """The raw stream of the `wrappers` golden case's scripted env: obs [T+1, O], reward, term, trunc,
    is_reset [T]."""
    raw = np.zeros((T + 1, O), np.float32)
    r, te, tr, rs = (np.zeros(T, np.float32) for _ in range(4))
    lib().orc_wrappers_script(C.c_int(O), C.c_int(T), C.c_int(reset_at), fp(raw), fp(r), fp(te), fp(tr), fp(rs))
    return raw, r, te, tr, rs


class SynthEnv:
    """Oracle synthetic vector env (SeqVectorEnv + RecordEpisodeStatistics semantics); with
    wrappers=True the PPO trainer's wrapper chain (ppo:41-49) sits on top, like make_env."""

    def __init__(self, E, O, A, wrappers=False, gamma=0.99):
        self.wrap = VecWrappers(E, O, gamma) if wrappers else None
        self.E, self.O, self.A = E, O, A
        self.q = np.zeros((E, O), np.float32); self.t = np.zeros(E, np.int32)
        self.ar = np.zeros(E, np.int32); self.rseed = np.zeros(E, np.uint32); self.rcount = np.zeros(E, np.uint32)
        self.ep_ret = np.zeros(E, np.float32); self.ep_len = np.zeros(E, np.int32)
        self.s = EnvState(E, O, A, *[x.ctypes.data for x in (self.q, self.t, self.ar, self.rseed, self.rcount,
                                                             self.ep_ret, self.ep_len)])

    def reset(self, seed):
        obs = np.zeros((self.E, self.O), np.float32)
        lib().orc_env_reset(C.byref(self.s), C.c_int(seed), fp(obs))
        return self.wrap.reset(obs) if self.wrap else obs

    def step(self, actions, lo=-1.0, hi=1.0):
        E = self.E
        obs = np.zeros((E, self.O), np.float32)
        r = np.zeros(E, np.float32); te = np.zeros(E, np.float32); tr = np.zeros(E, np.float32)
        ir = np.zeros(E, np.float32); il = np.zeros(E, np.int32)
        is_reset = (self.ar != 0).astype(np.float32)  # next-step autoreset pending before this step
        lib().orc_env_step(C.byref(self.s), fp(f32(actions)), C.c_float(lo), C.c_float(hi), fp(obs), fp(r), fp(te),
                           fp(tr), fp(ir), fp(il))
        if self.wrap:
            obs, r = self.wrap.step(obs, r, te, is_reset)
        return obs, r, te, tr, ir, il
