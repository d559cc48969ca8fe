"""Byte batches (alphabets outside {A,C,G,T}) on the duo kernels against the byte-path strip kernels.

Times kernel ms (sw_last_stats) of C3-shaped batches (1024 pairs of 8192 by default) over a given
alphabet with option duo_raw = 1 (the duo kernels, penalty from the bytes) and duo_raw = 0 (the
byte-path strip kernels), and of the same-shaped ACGT batch (the DNA duo) for reference; checks
that both byte runs give the same scores.  One JSON line per alphabet.

    python tools/bench_raw.py [--pairs P] [--n N] [--reps R] [--alpha protein,bytes,acgtn] [--params 1,-1,1,1]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ALPHA = {"protein": b"ACDEFGHIKLMNPQRSTVWY", "acgtn": b"ACGTN", "bytes": bytes(range(256)), "acgt": b"ACGT"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1024)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--alpha", default="protein,bytes,acgtn,acgt")
    ap.add_argument("--params", default="1,-1,1,1")
    a = ap.parse_args()
    import concurrentproject_amd as sw
    prm = sw.Params(*[int(x) for x in a.params.split(",")])
    for name in a.alpha.split(","):
        al = np.frombuffer(ALPHA[name], np.uint8)
        rng = np.random.default_rng(a.n)
        pairs = [(al[rng.integers(0, len(al), a.n)], al[rng.integers(0, len(al), a.n)]) for _ in range(a.pairs)]
        cells = a.pairs * a.n * a.n
        out = {"alphabet": name, "pairs": a.pairs, "n": a.n, "params": a.params}
        scores = {}
        for raw in ((1, 0) if name != "acgt" else (1,)):
            sw.set_option("duo_raw", raw)
            ms = []
            for _ in range(a.reps + 1):
                sc = sw.score_batch(pairs, prm)
                st = sw.last_stats()
                ms.append(st["kernel_ms"])
            k = min(ms[1:])
            key = "duo" if raw else "strip"
            out[key] = {"kernel_ms": round(k, 4), "gcups": round(cells / k / 1e6, 1), "mode": st["mode"],
                        "W": st["W"], "variant": st["variant"], "dna": st["dna"]}
            scores[key] = sc
        sw.set_option("duo_raw", 1)
        if "strip" in scores:
            out["scores_equal"] = scores["duo"] == scores["strip"]
            out["speedup"] = round(out["strip"]["kernel_ms"] / out["duo"]["kernel_ms"], 3)
        out["max_score"] = int(max(scores["duo"]))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
