#!/usr/bin/env python3
"""Generate the C5 golden (BASELINE.json configs[4]: one pair N = 2^20, seed 1048576).

TEST INFRASTRUCTURE (build container only).  Two independent CPU engines score the
same pair; the golden is committed only when they agree:

  --engine ref        the reference's OWN LazySmith (lazySmith.cpp:15-69), compiled in
                      place from /root/reference into oracle/_ref/libswref.so by
                      oracle/Makefile (`make -C oracle ref`); single thread, ~2 h.
  --engine wavefront  the oracle's pthread anti-diagonal restatement (sw_oracle.c
                      swo_wavefront, main.cpp:54-66 cell by cell), --threads T.

Each run writes tests/golden/c5_<engine>.json ({score, seconds, sha256}).  With
--merge, both results are compared and configs.json["C5"] is written.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

SEED, N = 1048576, 1 << 20


def sha(a, b):
    h = hashlib.sha256()
    h.update(np.asarray(a, np.uint8).tobytes()); h.update(b"|"); h.update(np.asarray(b, np.uint8).tobytes())
    return h.hexdigest()


def run(engine: str, threads: int) -> None:
    a, b = oracle.gen_pair(SEED, N)
    t0 = time.time()
    if engine == "ref":
        s = oracle.ref_score(a, b, which="lazy")
        if s is None:
            raise SystemExit("oracle/_ref/libswref.so missing: make -C oracle ref")
        src = "reference LazySmith (lazySmith.cpp:15-69) compiled from /root/reference, 1 thread"
    else:
        s = oracle.score_wavefront(a, b, threads=threads)
        src = "oracle swo_wavefront (sw_oracle.c, main.cpp:54-66 restated), %d threads" % threads
    dt = time.time() - t0
    out = {"seed": SEED, "N": N, "score": int(s), "seconds": round(dt, 1), "sha256": sha(a, b), "source": src}
    with open(os.path.join(HERE, "c5_%s.json" % engine), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)


def merge() -> None:
    """configs.json["C5"] from every engine result present; all must agree."""
    res = [json.load(open(os.path.join(HERE, "c5_%s.json" % e))) for e in ("ref", "wavefront")
           if os.path.exists(os.path.join(HERE, "c5_%s.json" % e))]
    assert res, "no C5 result yet"
    assert len({r["sha256"] for r in res}) == 1, "different pairs"
    assert len({r["score"] for r in res}) == 1, [r["score"] for r in res]
    path = os.path.join(HERE, "configs.json")
    cfg = json.load(open(path))
    cfg["C5"] = {"seed": SEED, "N": N, "score": res[0]["score"], "sha256": res[0]["sha256"],
                 "pinned_by": [r["source"] + " in %.0f s" % r["seconds"] for r in res]}
    with open(path, "w") as f:
        json.dump(cfg, f, indent=1)
    print("C5", res[0]["score"], cfg["C5"]["pinned_by"])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", choices=["ref", "wavefront"])
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--merge", action="store_true")
    args = ap.parse_args()
    if args.merge:
        merge()
    else:
        run(args.engine, args.threads)
