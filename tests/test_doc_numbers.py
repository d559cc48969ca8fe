"""CPU: README.md / DESIGN.md quote the headline numbers of the records they name -- the driver's newest
BENCH_rNN.json and this round's default bench line profiles/rNN_bench_c2.json (tools/check_doc_numbers.py)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_docs_quote_the_records():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_doc_numbers.py")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
