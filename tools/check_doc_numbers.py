#!/usr/bin/env python3
"""Check the headline numbers README.md and DESIGN.md quote against the records they come from.

    python tools/check_doc_numbers.py

1. The driver's newest record (BENCH_rNN.json at the repository root, NN the largest): README.md and
   DESIGN.md must name that file, and quote its C2 `ms_per_step` (3 decimals) and `value` (GCUPS, an
   integer) from `parsed`; where the record's stdout tail still holds the C5 affine sub-line, its
   `ms_per_step` too (1 decimal).  A record newer than the documents (the driver writes BENCH_rNN.json at
   the end of round NN, after the documents) is reported and checked as far as it goes.
2. This round's own default bench line (profiles/rNN_bench_c2.json for the newest NN present): README.md
   must quote every workload of its `summary` (bench.py headline_summary) -- ms_per_step at 3 decimals
   below 10 ms, 1 decimal above, and the GCUPS as an integer.
Exit status 1 on any mismatch."""
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fmt_ms(x):
    return ("%.3f" % x) if x < 10 else ("%.1f" % x)


def newest(pattern, rx):
    best = None
    for p in glob.glob(os.path.join(ROOT, pattern)):
        m = re.search(rx, os.path.basename(p))
        if m and (best is None or int(m.group(1)) > best[0]):
            best = (int(m.group(1)), p)
    return best


def main():
    docs = {name: open(os.path.join(ROOT, name)).read() for name in ("README.md", "DESIGN.md")}
    bad, ok = [], []
    rec = newest("BENCH_r*.json", r"BENCH_r(\d+)\.json")
    if rec is not None:
        nn, path = rec
        d = json.load(open(path))
        p = d.get("parsed") or {}
        name = os.path.basename(path)
        want = ["%s" % name]
        if p.get("ms_per_step") is not None:
            want.append(fmt_ms(p["ms_per_step"]) + " ms")
        if p.get("value") is not None:
            want.append("%d GCUPS" % round(p["value"]))
        m = re.search(r'"affine": \{"params": \[2, -3, 5, 2\], "ms_per_step": ([0-9.]+)', d.get("tail") or "")
        if m:
            want.append(fmt_ms(float(m.group(1))) + " ms")
        for doc, text in docs.items():
            missing = [w for w in want if w not in text]
            if missing:
                bad.append("%s does not quote %s: %s" % (doc, name, missing))
            else:
                ok.append("%s quotes %s: %s" % (doc, name, want))
    own = newest("profiles/r*_bench_c2.json", r"r(\d+)_bench_c2\.json")
    if own is not None:
        nn, path = own
        line = [json.loads(l) for l in open(path) if l.startswith("{")][-1]
        summ = line.get("summary") or {}
        want = []
        for key, row in summ.items():
            if isinstance(row, list) and len(row) == 3 and row[0] is not None:
                want.append(fmt_ms(row[0]) + " ms")
                if row[1] is not None:
                    want.append("%d GCUPS" % row[1])
        missing = [w for w in want if w not in docs["README.md"]]
        rel = os.path.relpath(path, ROOT)
        if missing:
            bad.append("README.md does not quote %s: %s" % (rel, missing))
        else:
            ok.append("README.md quotes %s: %d numbers" % (rel, len(want)))
    for o in ok:
        print("ok", o)
    for b in bad:
        print("FAIL", b)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
