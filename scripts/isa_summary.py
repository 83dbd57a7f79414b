#!/usr/bin/env python3
"""Summarise one kernel of a hipcc --save-temps gfx950 .s file: run-length counts of MFMA / LDS /
VALU instructions between waits, barriers, branches and memory ops (scheduling review aid)."""
import re
import sys


def main(path, kernel, limit=100000):
    s = open(path).read()
    i = s.index(kernel + ":")
    e = s.index(".Lfunc_end", i)
    out = []

    def bump(tag):
        if out and out[-1][0] == tag:
            out[-1][1] += 1
        else:
            out.append([tag, 1])
    for ln in s[i:e].split("\n"):
        t = ln.strip()
        if not t or t.startswith(";") or t.startswith("."):
            if t.startswith(".LBB"):
                out.append([t.split()[0], 0])
            continue
        op = t.split()[0]
        if "mfma" in op:
            bump("MFMA")
        elif op.startswith("ds_read") or op.startswith("ds_load"):
            bump("DSR")
        elif op.startswith("ds_write") or op.startswith("ds_store"):
            bump("DSW")
        elif op.startswith(("s_waitcnt", "s_barrier", "s_cbranch", "s_branch")):
            out.append([t, 0])
        elif op.startswith(("global_", "buffer_", "scratch_")):
            bump(op)
        elif op.startswith("v_"):
            bump("VALU")
        elif op.startswith("s_"):
            bump("SALU")
    for tag, n in out[:limit]:
        print(f"{tag} x{n}" if n else tag)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 100000)
