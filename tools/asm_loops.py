#!/usr/bin/env python3
"""Per-kernel innermost-loop instruction census of a hipcc -save-temps .s file.

    python tools/asm_loops.py build/asm/sw_kernels-hip-amdgcn-amd-amdhsa-gfx950.s [filter]
"""
import collections
import re
import sys


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


def loops(body):
    """Innermost loops: from a 'Loop Header' label to the backward branch to it."""
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_cbranch\w*\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            s = labels[m.group(1)]
            seg = body[s:i + 1]
            if any(re.match(r"^\.LBB\S+:", x) and "Loop Header" in "".join(body[j] for j in range(s, min(s + 3, len(body)))) for x in seg[:1]):
                pass
            inner = not any(re.match(r"^\s+s_cbranch\w*\s+(\.LBB\S+)", x) and x.split()[-1] in labels
                            and s < labels[x.split()[-1]] < i for x in seg[1:-1])
            if inner:
                yield s, i, seg


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(path):
        if filt not in name:
            continue
        best = None
        for s, e, seg in loops(body):
            ins = [x.split()[0] for x in seg if re.match(r"^\s+[vsgbd][a-z_0-9]+", x)]
            v = [x for x in ins if x.startswith("v_")]
            if best is None or len(v) > len(best[1]):
                best = (ins, v)
        if best:
            c = collections.Counter(best[0])
            print("%s  VALU=%d SALU=%d  %s" % (name, len(best[1]), sum(1 for x in best[0] if x.startswith("s_")),
                                                 ", ".join("%s:%d" % kv for kv in c.most_common(10))))


if __name__ == "__main__":
    main()
