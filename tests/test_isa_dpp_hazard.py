"""Build-time check of the DPP read-after-VALU-write hazard in k_rollout_v.

`fmac_bc` (csrc/ppo_rollout.hip) issues `v_fmac_f32_dpp acc, x, w row_newbcast:K` from inline asm.
The DPP source x must not be written by a VALU instruction within the two wait states before the
DPP instruction (CDNA3/4 ISA, "manually inserted wait states"): the compiler's hazard recognizer
does not see inside asm strings, so if register allocation ever put a VALU copy of x right before a
chain, the layer results would be silently wrong. This test disassembles the gfx950 code object of
the built ppo_rollout.o and checks every v_fmac_f32_dpp against the instructions before it.
No GPU needed.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "ppo.cpp_amd", "build", "ppo_rollout.o")
LLVM = "/opt/rocm/lib/llvm/bin"


def _vregs(tok):
    """VGPR indices named by one operand token (v7, v[8:11]); empty for anything else."""
    m = re.fullmatch(r"v(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _disassemble(tmp_path):
    if not os.path.exists(OBJ):
        pytest.skip("ppo.cpp_amd/build/ppo_rollout.o not built (run __graft_entry__.build())")
    if not os.path.exists(os.path.join(LLVM, "llvm-objdump")):
        pytest.skip("llvm-objdump not available")
    obj = tmp_path / "r.o"
    shutil.copy(OBJ, obj)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", str(obj)], cwd=tmp_path, check=True,
                   capture_output=True)
    dev = [p for p in os.listdir(tmp_path) if p.endswith("gfx950")]
    assert dev, os.listdir(tmp_path)
    out = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", str(tmp_path / dev[0])],
                         check=True, capture_output=True, text=True).stdout
    return out.splitlines()


def test_no_valu_write_to_a_dpp_source_within_two_wait_states(tmp_path):
    lines = _disassemble(tmp_path)
    insts = []  # (text, is_label)
    for ln in lines:
        t = ln.split("//")[0].strip()
        if not t:
            continue
        if t.endswith(">:") or t.endswith(":"):
            insts.append((t, True))
        elif re.match(r"^[sv]_|^ds_|^buffer_|^global_|^scratch_|^flat_", t):
            insts.append((t, False))
    n_dpp = 0
    bad = []
    for i, (t, lab) in enumerate(insts):
        if lab or not t.startswith("v_fmac_f32_dpp"):
            continue
        n_dpp += 1
        ops = [o.strip() for o in t.split(None, 1)[1].split(",")]
        src0 = _vregs(ops[1].split()[0])
        assert src0, t
        waits, j = 0, i - 1
        while waits < 2 and j >= 0:
            pt, plab = insts[j]
            if plab:  # a block boundary inside the window: the predecessor is not known statically
                bad.append((t, "label within two wait states: " + pt))
                break
            op = pt.split()[0]
            if op == "s_nop":
                waits += int(pt.split()[1], 0) + 1
            else:
                if op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane", "v_readfirstlane")):
                    dst = _vregs(pt.split(None, 1)[1].split(",")[0].strip()) if len(pt.split()) > 1 else set()
                    if dst & src0:
                        bad.append((t, pt))
                        break
                waits += 1
            j -= 1
    assert n_dpp >= 2 * (17 + 256), n_dpp  # k_rollout_v<1> and <2>: layer 1 (OP positions) + layer 2 chains
    assert not bad, bad[:5]
