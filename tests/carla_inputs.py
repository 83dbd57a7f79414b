"""Deterministic CaRL inputs and parameters, identical to oracle/ref_harness.cpp's carla_act case
(so the fixture stores outputs only): u(stream, i) = ((mix32(mix32(stream * 0x9E3779B1) ^ i) >> 8)
+ 0.5) * 2^-24 with mix32 the murmur3 finalizer."""
import ctypes as C

import numpy as np

import oracle_lib as O

N, CH, HW, NM, NV, A, BETA_MIN = 3, 15, 192, 8, 3, 2, 1.0
MAX_T = 40
NCONV = 6


class CarlaLayout(C.Structure):
    _fields_ = [("C", C.c_int), ("IH", C.c_int), ("IW", C.c_int), ("NM", C.c_int), ("NV", C.c_int), ("A", C.c_int),
                ("P", C.c_long), ("hi", C.c_long), ("lo", C.c_long),
                ("conv_w", C.c_long * NCONV), ("conv_b", C.c_long * NCONV),
                ("conv_ic", C.c_int * NCONV), ("conv_oc", C.c_int * NCONV), ("conv_k", C.c_int * NCONV),
                ("conv_s", C.c_int * NCONV), ("conv_ih", C.c_int * NCONV), ("conv_iw", C.c_int * NCONV),
                ("conv_oh", C.c_int * NCONV), ("conv_ow", C.c_int * NCONV),
                ("lin_w", C.c_long * 2), ("lin_b", C.c_long * 2), ("st_w", C.c_long * 2), ("st_b", C.c_long * 2),
                ("v_w", C.c_long * 3), ("v_b", C.c_long * 3), ("pi_w", C.c_long * 2), ("pi_b", C.c_long * 2),
                ("mu_w", C.c_long), ("mu_b", C.c_long), ("sg_w", C.c_long), ("sg_b", C.c_long),
                ("ntensors", C.c_int), ("t_off", C.c_long * MAX_T), ("t_len", C.c_long * MAX_T),
                ("t_grad", C.c_int * MAX_T)]


def mix32(h):
    h = np.asarray(h, np.uint32).copy()
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x85EBCA6B)
    h ^= h >> np.uint32(13)
    h *= np.uint32(0xC2B2AE35)
    h ^= h >> np.uint32(16)
    return h


def hbits(stream, n):
    with np.errstate(over="ignore"):
        s = mix32(np.uint32((stream * 0x9E3779B1) & 0xFFFFFFFF))
        return mix32(s ^ np.arange(n, dtype=np.uint32))


def hunif(stream, n, lo, hi):
    u = ((hbits(stream, n) >> np.uint32(8)).astype(np.float32) + np.float32(0.5)) * np.float32(5.9604644775390625e-8)
    return (np.float32(lo) + np.float32(hi - lo) * u).astype(np.float32)


def layout(C_=CH, IH=HW, IW=HW, NM_=NM, NV_=NV, A_=A):
    L = CarlaLayout()
    assert O.lib().orc_carla_layout_init(C.byref(L), C_, IH, IW, NM_, NV_, A_) == 0
    return L


def params(L):
    """Tensor t of named_parameters() from stream 1000 + t: weights U(+-sqrt(6 / fan_in)), biases
    U(+-0.1), action space [-1, 1] (ref_harness.cpp carla_act)."""
    p = np.zeros(L.P, np.float32)
    p[L.hi], p[L.lo] = 1.0, -1.0
    shapes = {}
    for i in range(NCONV):
        shapes[L.conv_w[i]] = L.conv_ic[i] * L.conv_k[i] * L.conv_k[i]
    for w, fan in ((L.lin_w[0], 1280), (L.lin_w[1], 512), (L.st_w[0], L.NM), (L.st_w[1], 256), (L.v_w[0], 256 + L.NV),
                   (L.v_w[1], 256), (L.v_w[2], 256), (L.pi_w[0], 256), (L.pi_w[1], 256), (L.mu_w, 256), (L.sg_w, 256)):
        shapes[w] = fan
    for t in range(L.ntensors):
        o, n = L.t_off[t], L.t_len[t]
        if o in (L.hi, L.lo):
            continue
        if o in shapes:
            a = np.float32(np.sqrt(np.float32(6.0) / np.float32(shapes[o])))
            p[o:o + n] = hunif(1000 + t, n, -a, a)
        else:
            p[o:o + n] = hunif(1000 + t, n, -0.1, 0.1)
    return p


def inputs(n=N):
    bev = (hbits(1, n * CH * HW * HW) >> np.uint32(24)).astype(np.uint8).reshape(n, CH, HW, HW)
    meas = hunif(2, n * NM, -1.0, 1.0).reshape(n, NM)
    vmeas = hunif(3, n * NV, -1.0, 1.0).reshape(n, NV)
    act = hunif(4, n * A, -0.98, 0.98).reshape(n, A)
    return bev, meas, vmeas, act


def oracle_forward(L, p, bev, meas, vmeas, mode, act=None, seed=1, rank=0, env_base=0, step_id=0):
    lib = O.lib()
    n = bev.shape[0]
    out = {k: np.zeros(s, np.float32) for k, s in (("action", (n, L.A)), ("logprob", n), ("entropy", n),
                                                   ("value", n), ("alpha", (n, L.A)), ("beta", (n, L.A)),
                                                   ("features", (n, 256)))}
    a = np.ascontiguousarray(act if act is not None else np.zeros((n, L.A), np.float32), np.float32)
    lib.orc_carla_forward(C.byref(L), O.fp(p), C.c_float(BETA_MIN), n, O.fp(np.ascontiguousarray(bev)),
                          O.fp(np.ascontiguousarray(meas)), O.fp(np.ascontiguousarray(vmeas)), mode, O.fp(a),
                          C.c_uint64(seed), rank, C.c_long(env_base), C.c_long(step_id),
                          *[O.fp(out[k]) for k in ("action", "logprob", "entropy", "value", "alpha", "beta",
                                                   "features")])
    return out
