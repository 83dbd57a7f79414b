"""One HIP runtime per process (include/ppo_hip.h ppo_runtime_check). libppo_hip.so links
/opt/rocm's libamdhip64.so.7; the PyTorch-ROCm wheel bundles its own copy, which its libraries load
by another name. torch first: libppo_hip.so binds to the runtime already mapped (one runtime).
libppo_hip.so first: `import torch` maps a second runtime; the library must say so on its next
runtime-initialising call and end the process with status 70 at exit instead of the corrupted-heap
abort (exit 134) that two runtimes tearing each other down produce. Fresh subprocesses, CPU only
(no device call is made)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ppo.cpp_amd", "lib", "libppo_hip.so")
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libppo_hip.so not built")

PROBE = r"""
import ctypes, sys
order = sys.argv[1]
if order == "torch_first":
    import torch  # noqa: F401
lib = ctypes.CDLL(sys.argv[2], mode=ctypes.RTLD_GLOBAL)
if order == "lib_first":
    import torch  # noqa: F401
lib.ppo_last_error.restype = ctypes.c_char_p
rc = lib.ppo_runtime_check()
print("rc", rc, lib.ppo_last_error().decode() if rc else "", flush=True)
"""


def run(order):
    return subprocess.run([sys.executable, "-c", PROBE, order, LIB], capture_output=True, text=True, timeout=240)


def test_torch_first_maps_one_runtime():
    r = run("torch_first")
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("rc 0"), r.stdout


def test_library_first_is_detected_and_exits_cleanly():
    r = run("lib_first")
    assert "two HIP runtimes" in r.stdout, (r.stdout, r.stderr[-2000:])
    assert r.returncode == 70, (r.returncode, r.stderr[-2000:])
    assert "exiting (70)" in r.stderr
