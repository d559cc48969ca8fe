#!/usr/bin/env python3
"""Static census of flow3's generated chunk loops (concurrentproject_amd/csrc/sw_flow3_loops.inc
and sw_flow3r_loops.inc): for every (C, role) block, the instructions of the loop's fast path
-- from `L_loop` to its back-edge branch, without the out-of-line slow paths -- by class,
per chunk.

    python tools/flow3_census.py [--json]

Classes: step (the W2 step's VALU: 9 per step), other VALU, SALU (scalar ALU and branches,
not s_nop / s_waitcnt), s_nop (wait states), s_waitcnt, DS (LDS), VMEM (buffer loads/stores).
"""
from __future__ import annotations

import json
import os
import re
import sys

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "concurrentproject_amd", "csrc")
FILES = ("sw_flow3_loops.inc", "sw_flow3r_loops.inc")
HEAD = re.compile(r"f3r?_loop<([^>]*)>")
INSN = re.compile(r'^\s*"([a-z_0-9]+)')


def blocks(path):
    """[(signature, [instruction mnemonics + operands of the fast loop])]"""
    out, sig, body, inloop = [], None, [], False
    for line in open(path):
        m = HEAD.search(line)
        if m and "template" in line:
            sig, body, inloop = m.group(1).replace(" ", ""), [], False
            continue
        s = line.strip()
        if not s.startswith('"'):
            continue
        text = s[1:].split("\\n")[0]
        if text.startswith("L_loop_%=:"):
            inloop = True
            continue
        if inloop:
            body.append(text)
            if re.match(r"s_cbranch_\w+ L_loop_%=", text):
                inloop = False
                out.append((sig, body))
    return out


def classify(insn):
    op = insn.split()[0]
    if op.endswith(":"):
        return None   # a label inside the fast path
    if op == "s_nop":
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith("buffer_") or op.startswith("global_"):
        return "vmem"
    if op.startswith("v_"):
        return "valu"
    return "other"


def census(sig, body):
    cnt = {"valu": 0, "salu": 0, "s_nop": 0, "s_nop_cycles": 0, "waitcnt": 0, "ds": 0, "vmem": 0, "other": 0}
    max3 = 0
    for insn in body:
        k = classify(insn)
        if k is None:
            continue
        cnt[k] += 1
        if k == "s_nop":
            cnt["s_nop_cycles"] += int(insn.split()[1], 0) + 1
        if insn.startswith("v_max3"):
            max3 += 1
    steps = max3 // 3               # the W2 step has 3 max3
    C = int(sig.split(",")[0]) if sig.split(",")[0].isdigit() else 64
    chunks = max(1, steps // C)
    per = {k: round(v / chunks, 2) for k, v in cnt.items()}
    per["step_valu"] = 9 * C
    per["extra_valu"] = round(cnt["valu"] / chunks - 9 * C, 2)
    return {"loop": sig, "C": C, "steps_per_iteration": steps, "chunks_per_iteration": chunks, "per_chunk": per}


def main():
    rows = []
    for f in FILES:
        for sig, body in blocks(os.path.join(CSRC, f)):
            r = census(sig, body)
            r["file"] = f
            rows.append(r)
    if "--json" in sys.argv:
        print(json.dumps(rows, indent=1))
        return
    print("%-22s %-22s %5s %6s %6s %6s %6s %5s %5s" % ("file", "loop <C,IN,OUT>", "steps", "xVALU", "SALU", "s_nop",
                                                       "wait", "DS", "VMEM"))
    for r in rows:
        p = r["per_chunk"]
        print("%-22s %-22s %5d %6.1f %6.1f %6.1f %6.1f %5.1f %5.1f" % (
            r["file"], r["loop"], r["steps_per_iteration"], p["extra_valu"], p["salu"], p["s_nop"], p["waitcnt"],
            p["ds"], p["vmem"]))
    print("(per chunk; xVALU = VALU beyond the 9 per step of the W2 body)")


if __name__ == "__main__":
    main()
