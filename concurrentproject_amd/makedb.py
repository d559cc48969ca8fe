"""``python -m concurrentproject_amd.makedb in.fasta out.swdb``: the binary
database of a FASTA file (the ``makedb`` step of the reference's timing.sh:6,
CUDASW++4's tool there; here include/algoGPU.h ``sw_db_save``)."""
import argparse
import sys

from .db import Database


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="makedb", description=__doc__)
    ap.add_argument("fasta")
    ap.add_argument("out")
    a = ap.parse_args(argv)
    with Database.open(a.fasta) as db:
        db.save(a.out)
        print("%d records, %d residues -> %s" % (len(db), db.residues, a.out), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
