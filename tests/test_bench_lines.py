"""CPU: every committed bench line of this round (profiles/r06*_bench_*.json) carries a
counter-derived roofline whose `frac` / `achieved` match the profiles/pmc_*.json it names
(same sha256) to 3 digits, and whose config.kernel_fn is the kernel that profile counted
(tools/check_bench_lines.py, strict mode)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_committed_bench_lines_match_their_profiles():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_bench_lines.py")], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok ") >= 4, r.stdout
