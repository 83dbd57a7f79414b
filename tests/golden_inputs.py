"""Deterministic inputs of the round-2 golden cases (oracle/ref_harness.cpp width_cases()).

The fixtures store inputs and outputs; the agent parameters and the long-GAE inputs are drawn
from hash streams instead, restated here:
  u(stream, i) = ((mix32(mix32(stream * 0x9E3779B1) ^ i) >> 8) + 0.5) * 2^-24   (carla_inputs.py)
  value        = lo + (hi - lo) * u, all float32
"""
import numpy as np

from carla_inputs import hbits


def hunif32(stream, n, lo, hi):
    """ref_harness.cpp hunif(): lo + (hi - lo) * u evaluated in float32."""
    u = ((hbits(stream, n) >> np.uint32(8)).astype(np.float32) + np.float32(0.5)) * np.float32(5.9604644775390625e-8)
    lo32, hi32 = np.float32(lo), np.float32(hi)
    return (lo32 + (hi32 - lo32) * u).astype(np.float32)


def hash_params(L, base, hi=1.0, lo=-1.0):
    """ref_harness.cpp hash_params(): tensor t of named_parameters() from stream base + t."""
    fan = {}
    for tr in (L.critic, L.actor):
        fan[tr[0]] = L.O
        fan[tr[4]] = L.H
    for off in (L.cW3, L.aW3, L.bW3):
        if off >= 0:
            fan[off] = L.H
    gammas = set()
    if L.kind == 1:
        for tr in (L.critic, L.actor):
            gammas.update((tr[2], tr[6]))
    p = np.zeros(L.P, np.float32)
    for t in range(L.ntensors):
        o, n, s = L.t_off[t], L.t_len[t], base + t
        if o == L.hi:
            v = np.float32([hi])
        elif o == L.lo:
            v = np.float32([lo])
        elif o == L.omean:
            v = hunif32(s, n, -0.1, 0.1)
        elif o == L.ostd:
            v = hunif32(s, n, 0.8, 1.5)
        elif o == L.logstd:
            v = hunif32(s, n, -0.7, -0.3)
        elif o in gammas:
            v = hunif32(s, n, 0.8, 1.2)
        elif o in fan:
            a = np.sqrt(np.float32(3.0) / np.float32(fan[o])).astype(np.float32)
            v = hunif32(s, n, -a, a)
        else:
            v = hunif32(s, n, -0.1, 0.1)
        p[o:o + n] = v
    return p


def column_fnv(a):
    """FNV-1a 64 of each column's float32 bit patterns, rows in order (ref_harness.cpp column_fnv)."""
    b = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    h = np.full(b.shape[1], 14695981039346656037, np.uint64)
    prime = np.uint64(1099511628211)
    with np.errstate(over="ignore"):
        for t in range(b.shape[0]):
            h ^= b[t]
            h *= prime
    return h.view(np.int64)


def gae_long_inputs(T=2048, E=1024):
    """Inputs of the gae_long case (streams 11-15)."""
    n = T * E
    rewards = hunif32(11, n, -1.0, 1.0).reshape(T, E)
    values = hunif32(12, n, -1.0, 1.0).reshape(T, E)
    dones = (hunif32(13, n, 0.0, 1.0) < np.float32(0.002)).astype(np.float32).reshape(T, E)
    dones[0] = 1.0
    dones[T - 1, :E // 2] = 1.0
    next_value = hunif32(14, E, -1.0, 1.0)
    next_done = (hunif32(15, E, 0.0, 1.0) < np.float32(0.5)).astype(np.float32)
    return rewards, values, dones, next_value, next_done


def wrapper_script(O=5, T=200, reset_at=120):
    """The scripted env of the `wrappers` case: per call c (reset or step) the raw obs row,
    the raw step reward and the termination / truncation flags."""
    def obs(c):
        i = np.arange(O)
        u = hunif32(30, (c + 1) * O, 0.0, 1.0)[c * O:(c + 1) * O]
        lo = i.astype(np.float32) - np.float32(2.0)
        hi = i.astype(np.float32) + np.float32(3.0)
        return (lo + (hi - lo) * u).astype(np.float32)
    return obs
