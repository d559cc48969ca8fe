"""``python -m concurrentproject_amd.align --query q.fa --db sp.swdb [--top K]``:
every query record scored against every database record on the GPU (the
``align`` step of the reference's timing.sh:7, CUDASW++4's tool there).

Prints, per query, its K best hits as tab-separated lines
``query_index  query_header  rank  score  db_index  db_header``; the search's
cells, time and GCUPS go to stderr.  Scores are the reference's byte-equality
affine scores (main.cpp:28-66) with --params MATCH,MISMATCH,G_INIT,G_EXT."""
import argparse
import sys
import time

import numpy as np

from . import Params, set_params
from .db import Database


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="align", description=__doc__)
    ap.add_argument("--query", required=True, help="FASTA file (or a makedb file) of queries")
    ap.add_argument("--db", required=True, help="FASTA file or a makedb file")
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--params", default="1,-1,1,1", help="MATCH,MISMATCH,G_INIT,G_EXT")
    a = ap.parse_args(argv)
    set_params(Params(*(int(x) for x in a.params.split(","))))
    with Database.open(a.db) as db, Database.open(a.query) as qs:
        lens = db.lengths()
        t0 = time.perf_counter()
        scores = db.search_db(qs)
        dt = time.perf_counter() - t0
        cells = int(qs.lengths().sum()) * int(lens.sum())
        out = sys.stdout
        for q in range(len(qs)):
            qh = qs.header(q)
            sc = scores[q]
            order = np.lexsort((np.arange(len(sc)), -sc.astype(np.int64)))[:a.top]
            for r, i in enumerate(order):
                out.write("%d\t%s\t%d\t%d\t%d\t%s\n" % (q, qh, r + 1, int(sc[i]), int(i), db.header(int(i))))
        print("%d queries x %d records: %.3e cells in %.3f s = %.2f GCUPS"
              % (len(qs), len(db), cells, dt, cells / max(dt, 1e-12) / 1e9), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
