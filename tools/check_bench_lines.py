#!/usr/bin/env python3
"""Check committed bench lines against the counter profiles they were computed from.

    python tools/check_bench_lines.py [profiles/r06*_bench_*.json ...]

For every bench JSON line (the top-level roofline and the nested batch_c3 / batch_c4
rooflines) whose roofline names a profiles/pmc_*.json and carries its sha256
(`pmc_sha256`, bench.py): recompute
    achieved = valu_insts_per_launch * 64 / kernel time, frac = achieved / peak
from that file and the line's own kernel time, and require the line's values to
match to 3 significant digits.  A line whose profile file has changed since (another
sha256) is reported STALE; a line of this round (the default set) must be neither
stale nor carry frac: null.  Exit status 1 on any failure."""
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 256 * 4 * 32 * 2.4e9 / 1e12


def lines_of(path):
    out = []
    for l in open(path):
        l = l.strip()
        if l.startswith("{"):
            try:
                out.append(json.loads(l))
            except ValueError:
                pass
    return out


def rooflines(line):
    """(label, roofline, kernel ms, kernel_fn) of a bench line and its nested lines (the batched
    config, the affine step, the C5 extras)."""
    if "roofline" in line and "kernel_ms_per_launch" in line:
        yield "main", line["roofline"], line["kernel_ms_per_launch"], (line.get("config") or {}).get("kernel_fn")
    for key in ("batch_c3", "batch_c4", "affine_step"):
        sub = line.get(key)
        if isinstance(sub, dict) and "roofline" in sub:
            yield key, sub["roofline"], sub["kernel_ms_per_launch"], sub.get("kernel_fn")
        aff = (sub or {}).get("affine_step") if key != "affine_step" and isinstance(sub, dict) else None
        if isinstance(aff, dict) and "roofline" in aff:
            yield key + ".affine_step", aff["roofline"], aff["kernel_ms_per_launch"], aff.get("kernel_fn")
    for key in ("linear", "affine"):
        sub = (line.get("c5") or {}).get(key)
        if isinstance(sub, dict) and "roofline" in sub:
            yield "c5." + key, sub["roofline"], sub["kernel_ms_per_launch"], sub.get("kernel_fn")


def check(path, strict):
    bad = []
    for line in lines_of(path):
        for label, rf, kms, fn in rooflines(line):
            src = rf.get("source") or ""
            if not src.startswith("profiles/pmc_"):
                if strict:
                    bad.append("%s %s: no counter profile (%s)" % (path, label, src))
                continue
            pmc = os.path.join(ROOT, src)
            if not os.path.exists(pmc):
                bad.append("%s %s: %s missing" % (path, label, src))
                continue
            sha = hashlib.sha256(open(pmc, "rb").read()).hexdigest()
            if rf.get("pmc_sha256") != sha:
                if strict:
                    bad.append("%s %s: STALE (%s changed since the line was taken)" % (path, label, src))
                continue
            prof = json.load(open(pmc))
            # the kernel the line says it timed is the one the profile counted
            if fn is not None and "::" + fn + "<" not in prof["kernel"] and "::" + fn + "(" not in prof["kernel"]:
                bad.append("%s %s: config kernel_fn %s but %s profiles %s" % (path, label, fn, src, prof["kernel"]))
                continue
            ach = prof["valu_insts_per_launch"] * 64 / (kms * 1e-3) / 1e12
            frac = ach / PEAK
            if rf.get("frac") is None or abs(rf["frac"] - frac) > 0.0005 * max(1.0, frac) + 1e-4 \
                    or abs(rf["achieved"] - ach) > 0.001 * ach + 1e-3:
                bad.append("%s %s: frac %s / achieved %s, recomputed %.4f / %.3f"
                           % (path, label, rf.get("frac"), rf.get("achieved"), frac, ach))
            else:
                print("ok %s %s: frac %.4f (%s)" % (os.path.relpath(path, ROOT), label, frac, src))
    return bad


def main():
    args = sys.argv[1:]
    strict = not args
    paths = args or sorted(glob.glob(os.path.join(ROOT, "profiles", "r06*_bench_*.json")))
    bad = []
    for p in paths:
        bad += check(p, strict)
    for b in bad:
        print("FAIL", b)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
