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
    for h in ("ppo_hip.h", "ppo_synth_env.h", "ppo_carla.h", "ppo_pth.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*[A-Za-z_][\w\s\*]*?\b((?:ppo|psyn)_\w+)\s*\(", src, flags=re.M):
            if "static" not in m.group(0):  # header-only helpers (static inline layout initialisers)
                names.append(m.group(1))
    return sorted(set(names))


def test_headers_declare_the_boundary():
    names = declared_functions()
    for required in ("ppo_create", "ppo_get_action_and_value", "ppo_rollout_act", "ppo_compute_gae", "ppo_update",
                     "ppo_comm_init", "psyn_step"):
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
