"""CPU: generated kernel sources are in sync with their generators."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flow3_loops_in_sync():
    """concurrentproject_amd/csrc/sw_flow3_loops.inc is what tools/gen_flow3.py writes."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_flow3.py"), "--check"])
    assert r.returncode == 0, "run: python tools/gen_flow3.py"
