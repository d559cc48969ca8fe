#!/usr/bin/env python3
"""Chunk-loop census of a flow2 kernel in a hipcc -save-temps .s file (tools only).

    python tools/asm_chunks.py <file.s> <kernel-name-filter> [min_valu]

Every backward branch whose range holds >= min_valu VALU instructions is a chunk
loop (one per in/out role of the strip: dispatch_kinds instantiates the step loop
per role).  Prints, per loop, the VALU / SALU / s_nop / s_waitcnt / DS / VMEM
counts of the whole range (slow-path poll loops included: they sit inside it but
run only when an inflow is late) and the step-instruction share."""
import collections
import re
import sys

STEP = ("v_max3_i32", "v_add_u32_sdwa", "v_sub_u32_e64", "v_mov_b32_dpp", "v_add_u32_dpp", "v_perm_b32")


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end"):
                yield cur, body
                cur = None
            else:
                body.append(line.rstrip("\n"))


def main():
    path, filt = sys.argv[1], sys.argv[2]
    minv = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    for name, body in kernels(path):
        if filt not in name:
            continue
        labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\S+):", l)] if m}
        print(name)
        for i, l in enumerate(body):
            m = re.match(r"^\s+s_cbranch\w*\s+(\.LBB\S+)", l) or re.match(r"^\s+s_branch\s+(\.LBB\S+)", l)
            if not m or m.group(1) not in labels or labels[m.group(1)] >= i:
                continue
            seg = body[labels[m.group(1)]:i + 1]
            ins = [x.split()[0] for x in seg if re.match(r"^\s+[vsdgb][a-z_0-9]+", x)]
            v = [x for x in ins if x.startswith("v_")]
            if len(v) < minv:
                continue
            c = collections.Counter(ins)
            salu = sum(n for k, n in c.items() if k.startswith("s_") and k not in ("s_nop", "s_waitcnt"))
            ds = sum(n for k, n in c.items() if k.startswith("ds_"))
            vm = sum(n for k, n in c.items() if k.startswith(("buffer_", "global_")))
            step = sum(c[k] for k in STEP)
            other = sorted(((k, n) for k, n in c.items() if k.startswith("v_") and k not in STEP), key=lambda x: -x[1])
            print("  lines %d-%d VALU %d (step-class %d) SALU %d s_nop %d s_waitcnt %d DS %d VMEM %d  other VALU %s"
                  % (labels[m.group(1)], i, len(v), step, salu, c["s_nop"], c["s_waitcnt"], ds, vm, other[:8]))


if __name__ == "__main__":
    main()
