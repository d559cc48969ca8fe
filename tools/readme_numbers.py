#!/usr/bin/env python3
"""Rewrite the measured-numbers block of README.md (between the NUMBERS markers) from the records:
the driver's newest BENCH_rNN.json and this round's default bench line profiles/rNN_bench_c2.json
(its `summary`, bench.py headline_summary), so that tools/check_doc_numbers.py holds by construction.

    python tools/readme_numbers.py"""
import glob
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BEGIN, END = "<!-- NUMBERS BEGIN (tools/readme_numbers.py) -->", "<!-- NUMBERS END -->"
LABEL = {"c2": "C2, one pair N = 65536 (the headline `value`)", "c2_affine": "C2 with G_INIT != G_EXT (2, -3, 5, 2)",
         "c3": "C3, 1024 pairs N = 8192", "c3_affine": "C3 with (2, -3, 5, 2)", "c5": "C5, one pair N = 2^20",
         "c5_affine": "C5 with (2, -3, 5, 2)", "c2_lower": "C2 relabeled a, c, g, t (seven-letter kernels)",
         "c5_lower": "C5 relabeled a, c, g, t (seven-letter ring kernel)",
         "c3_lower": "C3 relabeled a, c, g, t (duo on raw bytes)"}


def fmt_ms(x):
    return ("%.3f" % x) if x < 10 else ("%.1f" % x)


def newest(pattern, rx):
    best = None
    for p in glob.glob(os.path.join(ROOT, pattern)):
        m = re.search(rx, os.path.basename(p))
        if m and (best is None or int(m.group(1)) > best[0]):
            best = (int(m.group(1)), p)
    return best


def block():
    out = [BEGIN]
    rec = newest("BENCH_r*.json", r"BENCH_r(\d+)\.json")
    if rec:
        d = json.load(open(rec[1]))
        p = d["parsed"]
        m = re.search(r'"affine": \{"params": \[2, -3, 5, 2\], "ms_per_step": ([0-9.]+)', d.get("tail") or "")
        out.append("Driver-timed, `%s` (the driver's own run of `bench.py` on a fresh MI355X at the end of round %d):"
                   % (os.path.basename(rec[1]), rec[0]))
        out.append("* C2: **%s ms** a step = **%d GCUPS**, parity ok;" % (fmt_ms(p["ms_per_step"]), round(p["value"])))
        if m:
            out.append("* C5 with (2, -3, 5, 2): %s ms (the part of the line the record's tail keeps);" % fmt_ms(float(m.group(1))))
        out.append("")
    own = newest("profiles/r*_bench_c2.json", r"r(\d+)_bench_c2\.json")
    if own:
        line = [json.loads(l) for l in open(own[1]) if l.startswith("{")][-1]
        s = line["summary"]
        out.append("This round's default bench line (`%s`, `bench.py --steps 10 --warmup 2` on one MI355X, every "
                   "score checked against its reference-pinned golden):" % os.path.relpath(own[1], ROOT))
        out.append("")
        out.append("| workload | ms per step | GCUPS | parity |")
        out.append("|---|---|---|---|")
        for k, lab in LABEL.items():
            if k in s:
                ms, g, par = s[k]
                out.append("| %s | %s ms | %d GCUPS | %s |" % (lab, fmt_ms(ms), g, par))
        if s.get("c3_int32_kernel_ms") is not None:
            out.append("")
            out.append("C3 on the int32 kernels (scores >= 2^16 take them): %s ms a launch on flow3's three-column step "
                       "with a pair per workgroup." % fmt_ms(s["c3_int32_kernel_ms"]))
    out.append(END)
    return "\n".join(out)


def main():
    path = os.path.join(ROOT, "README.md")
    text = open(path).read()
    b = block()
    if BEGIN in text:
        text = text[:text.index(BEGIN)] + b + text[text.index(END) + len(END):]
    else:
        text = text.rstrip() + "\n\n" + b + "\n"
    open(path, "w").write(text)
    print(b)


if __name__ == "__main__":
    main()
