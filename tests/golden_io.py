"""Loader for tests/golden/ fixtures written by oracle/ref_harness.cpp (data only)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_case(name):
    m = manifest()[name]
    out = {}
    for arr, info in m["arrays"].items():
        dt = np.float32 if info["dtype"] == "f32" else np.int64
        a = np.fromfile(os.path.join(GOLDEN, name, f"{arr}.{info['dtype']}"), dtype=dt)
        out[arr] = a.reshape(info["shape"]) if info["shape"] else a.reshape(())
    return m["meta"], out
