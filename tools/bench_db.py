"""Database-search rate (f-4): one query against a synthetic FASTA of ragged DNA (or protein) records.

Times ``Database.search`` (sw_db_search, synchronous: query H2D + one batch launch over every record + score D2H),
so the figure is host-API GCUPS, not kernel-only.  Records are uniform ACGT with lengths drawn uniformly from
[lo, hi]; the arena is uploaded to HBM by the first (untimed) search.  --alphabet protein: uniform over
the 20 amino-acid letters (SwissProt-style; the engine's byte path, duo kernels with option duo_raw = 1).

    python tools/bench_db.py [--records R] [--qlen Q] [--lo L] [--hi H] [--steps K] [--alphabet dna|protein]
                             [--opt k=v ...]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from concurrentproject_amd.db import Database  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=65536)
    ap.add_argument("--qlen", type=int, default=1024)
    ap.add_argument("--lo", type=int, default=256)
    ap.add_argument("--hi", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--alphabet", default="dna", choices=("dna", "protein"))
    ap.add_argument("--queries", type=int, default=0,
                    help="also time search_db over this many queries of qlen (pipelined on the database's stream)")
    ap.add_argument("--opt", action="append", default=[], help="engine option k=v (sw_set_option), repeatable")
    a = ap.parse_args()
    import concurrentproject_amd as sw
    for kv in a.opt:
        k, v = kv.split("=")
        sw.set_option(k, int(v))
    rng = np.random.default_rng(4)
    acgt = np.frombuffer(b"ACGT" if a.alphabet == "dna" else b"ACDEFGHIKLMNPQRSTVWY", dtype=np.uint8)
    lens = rng.integers(a.lo, a.hi + 1, size=a.records)
    parts = []
    for i, n in enumerate(lens):
        parts.append(b">r%d\n" % i + acgt[rng.integers(0, len(acgt), size=n)].tobytes() + b"\n")
    db = Database.from_fasta(b"".join(parts))
    q = acgt[rng.integers(0, len(acgt), size=a.qlen)]
    db.search(q)  # upload + warm
    t0 = time.perf_counter()
    for _ in range(a.steps):
        sc = db.search(q)
    dt = (time.perf_counter() - t0) / a.steps
    cells = int(lens.sum()) * a.qlen
    st = sw.last_stats()
    print(json.dumps({"metric": "db search GCUPS (host API, synchronous)", "alphabet": a.alphabet,
                      "kernel_ms": round(st.get("kernel_ms", -1), 3), "mode": st["mode"], "W": st["W"], "value": round(cells / dt / 1e9, 2),
                      "unit": "GCUPS", "ms_per_search": round(dt * 1e3, 3), "records": a.records,
                      "residues": int(lens.sum()), "qlen": a.qlen, "len_range": [a.lo, a.hi],
                      "max_score": int(sc.max())}))
    if a.queries:
        from concurrentproject_amd.db import Database as D
        qrecs = [("q%d" % k, acgt[rng.integers(0, len(acgt), size=a.qlen)].tobytes()) for k in range(a.queries)]
        qdb = D.from_records(qrecs)
        db.search_db(qdb)   # warm
        t0 = time.perf_counter()
        many = db.search_db(qdb)
        dm = (time.perf_counter() - t0) / a.queries
        t0 = time.perf_counter()
        one = [db.search(q) for _, q in qrecs]
        ds = (time.perf_counter() - t0) / a.queries
        print(json.dumps({"metric": "db search_db GCUPS (host API, pipelined queries)", "alphabet": a.alphabet,
                          "queries": a.queries, "ms_per_query": round(dm * 1e3, 3),
                          "value": round(cells / dm / 1e9, 2), "unit": "GCUPS",
                          "ms_per_query_one_by_one": round(ds * 1e3, 3),
                          "equal": all(many[k].tolist() == one[k].tolist() for k in range(a.queries))}))
        qdb.close()
    db.close()


if __name__ == "__main__":
    main()
