"""GPU parity: four and five columns per lane in flow3's ring mode (sw_flow3.hip sw_flow3r45_kernel,
chunk loops from tools/gen_flow3.py step_w; sw_engine.hip plan_w45): strips of 252 new columns, then
strips of 315, sized so that every four-strip group of a pair is resident in one round (option f2w = 4;
measured slower than three columns on C5, so not the automatic plan).  The linear-gap
step (main.cpp:54-66 at G_INIT == G_EXT, exact), bit-exact against the oracle
(lazySmith.cpp:15-69 restated), against the three-column kernel on the same inputs, and against the C5
golden on the automatic plan."""
import numpy as np
import pytest

from test_slab import _rand_dna, _similar

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _defaults(engine):
    def reset():
        engine.set_params(engine.Params())
        for k in ("W", "C", "blocks", "orient", "f2w", "f2_wgs"):
            engine.set_option(k, 0)
        engine.set_option("mode", -1)
        engine.set_option("ring", -1)
        engine.set_option("ring_rows", 4096)
        engine.set_option("linear", -1)
    reset()
    yield
    reset()


def _plan(n, blocks):
    """(strips of four columns, strips of five) of plan_w45 for n columns on `blocks` resident blocks."""
    g5 = max(0, (n - 1008 * blocks + 251) // 252)
    if g5 > blocks or n < 1024:
        return None
    s4, s5 = 4 * (blocks - g5), 0
    if 252 * (s4 - 1) + 256 < n:
        s5 = max(1, (n - 320 - 252 * s4 + 314) // 315 + 1)
    else:
        s4 = max(1, (n - 256 + 251) // 252 + 1)
    return s4, s5


def test_w45_ring_parity(engine, oracle_mod):
    """f2w = 4 forced with small grids: pairs cut into W4 strips only, W5 strips only and both (the
    W4 -> W5 hand-off), a grid too small for five columns (three then), rows around the 64-row
    chunks and 512-row rings; similar pairs put long diagonals through every strip edge."""
    rng = np.random.default_rng(45)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("ring", 1)
    engine.set_option("f2w", 4)
    op = oracle_mod.Params(1, -1, 1, 1)
    seen = set()
    for n, m, blocks, rows in ((1100, 700, 1, 512), (2000, 1000, 2, 512), (2100, 2049, 2, 512), (2300, 600, 2, 4096),
                               (3500, 1500, 3, 512), (3500, 3001, 2, 1024), (5000, 2000, 4, 512), (6000, 129, 5, 512),
                               (4100, 640, 4, 512)):
        a = _rand_dna(rng, n)
        b = _similar(rng, a, m) if rng.random() < 0.6 else _rand_dna(rng, m)
        engine.set_option("blocks", blocks)
        engine.set_option("ring_rows", rows)
        got = engine.score(a, b)
        exp = oracle_mod.score_linear(a, b, op)
        st = engine.last_stats()
        plan = _plan(n, blocks)
        if plan is None:
            assert not st["variant"] & 16384, (n, blocks, st)
        else:
            s4, s5 = plan
            assert st["variant"] & 16384 and st["variant"] & 4 and not st["variant"] & 8192, (n, blocks, st)
            assert st["items"] == (s4 + s5 + 3) // 4, (n, blocks, plan, st)
            seen.add(("w4" if s4 else "") + ("w5" if s5 else ""))
        assert got == exp, (n, m, blocks, rows, plan, got, exp)
    # W4 alone, W5 alone and the mixed cut were all exercised
    assert seen == {"w4", "w5", "w4w5"}, seen


def test_w45_matches_w3(engine):
    """A 2^17 pair on 128 blocks (a mixed W4 / W5 cut) and on the automatic plan (three columns,
    its 174 groups fit one round): the same score, also on the transposed problem."""
    N = 1 << 17
    a, b = engine.gen_pair(N, N)
    engine.set_option("ring", 1)
    w3 = engine.score(a, b)
    assert engine.last_stats()["variant"] & 8192 and not engine.last_stats()["variant"] & 16384
    engine.set_option("f2w", 4)
    engine.set_option("blocks", 128)
    assert _plan(N, 128)[1] > 0
    w45 = engine.score(a, b)
    st = engine.last_stats()
    assert st["variant"] & 16384 and st["blocks"] == 128, st
    assert w45 == w3 > 0
    engine.set_option("orient", 2)
    assert engine.score(a, b) == w3


def test_w45_config_c5(engine, golden):
    """C5 (N = 2^20, seed 1048576) with f2w = 4: 3832 strips of 252 columns and 264 of 315 in 1024
    groups, every one resident in one round (4 per CU); the golden score, O(N) edge state.  (The
    automatic plan keeps three columns per lane: faster)"""
    import torch
    c = golden("configs.json")["C5"]
    N = c["N"]
    a, b = engine.gen_pair(c["seed"], N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.set_option("f2w", 4)
    engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s.cuda_stream)
    engine.stream_status(s.cuda_stream)
    st = engine.last_stats()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    s4, s5 = _plan(N, 4 * cus)
    assert st["variant"] & 16384 and st["variant"] & 4, st
    assert st["items"] == (s4 + s5 + 3) // 4 == st["blocks"] <= 4 * cus, (st, s4, s5)
    assert st["boundary_bytes"] < 1 << 30, st
    assert score.item() == c["score"]
