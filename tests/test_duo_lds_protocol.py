"""CPU: the duo LDS kernel's hand-off protocol (tools/duo_lds_sim.py models
sw_duo_lds_kernel's rounds, rings, wrap buffer and progress-word arithmetic) has no
deadlock and never reads an overwritten slot, over random duo sequences with idle waves.
The round-end consumer report is what makes it deadlock-free: without it a producer waits
on a consumer that skipped rounds (the case the first GPU build timed out on)."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import duo_lds_sim  # noqa: E402


def test_random_duo_sequences():
    rng = random.Random(7)
    for t in range(150):
        duos = duo_lds_sim.random_duos(rng)
        ok, detail = duo_lds_sim.run(duos, t)
        assert ok, (duos, detail)


def test_idle_round_case_needs_round_end_report():
    duos = [(8, 2968), (7, 3530), (4, 684), (8, 416)]
    assert duo_lds_sim.run(duos, 0)[0]
    ok, detail = duo_lds_sim.run(duos, 0, round_end_report=False)
    assert not ok and detail[0] == "deadlock"
