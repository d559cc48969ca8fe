"""CPU: generated kernel sources are in sync with their generators."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flow3_loops_in_sync():
    """concurrentproject_amd/csrc/sw_flow3_loops.inc is what tools/gen_flow3.py writes."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_flow3.py"), "--check"])
    assert r.returncode == 0, "run: python tools/gen_flow3.py"


def test_flow3_census_fast_path():
    """The staged chunk loops' fast path (tools/flow3_census.py): at most 10 SALU per chunk in every
    role, no hazard s_nop (the generator emits none; the only s_nop 0 are gen_flow3.align8's 8-B
    alignment pads, at most 2 per chunk), and at most 32 VALU per chunk beyond the 9 per step of
    the W2 body (score perms and hand-off work included; profiles/r04_flow3_census.txt)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import flow3_census
    rows = [flow3_census.census(sig, body) for sig, body in
            flow3_census.blocks(os.path.join(flow3_census.CSRC, "sw_flow3_loops.inc"))]
    assert len(rows) == 18   # (C, half-chunk links) in (32, 0), (16, 0), (32, 1) x 6 roles
    for r in rows:
        p = r["per_chunk"]
        assert p["salu"] <= 10 and p["s_nop"] <= 2, r
        assert p["extra_valu"] <= 32, r
