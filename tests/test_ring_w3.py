"""GPU parity: three columns per lane in flow3's ring mode (option f2w = 3; sw_flow3.hip
sw_flow3r3_kernel / sw_flow3r3s_kernel, chunk loops from tools/gen_flow3.py step3): strips of 189
new columns overlapping by three, the linear-gap step (main.cpp:54-66 at G_INIT == G_EXT, exact,
DESIGN.md section 2) and the affine step (sw_flow3ra3_kernel / sw_flow3ra3s_kernel), bit-exact
against the oracle (lazySmith.cpp:15-69 restated), against the two-column kernels on the same
inputs, against the C5 golden, and as column slabs."""
import numpy as np
import pytest

from test_slab import _rand_dna, _run_threads, _similar

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


def _pairs(rng):
    # columns around the 189-column strips and the 756-column groups (1, 2, 4, 5, 8, 9 strips),
    # rows around the 64-row chunk pairs and 512-row rings
    out = []
    for n, m in ((190, 300), (192, 129), (193, 700), (381, 1000), (382, 513), (756, 1200), (759, 640),
                 (945, 2000), (1513, 1700), (1700, 2500), (3001, 900), (5000, 3000)):
        a = _rand_dna(rng, n)
        b = _similar(rng, a, m) if rng.random() < 0.5 else _rand_dna(rng, m)
        out.append((a, b))
    return out


def test_w3_ring_parity(engine, oracle_mod):
    """Ring mode forced on grids of 1, 2, 3 and 7 blocks with 512-row rings (many rounds, the
    wrap ring every round), three constant sets of the linear-gap step."""
    rng = np.random.default_rng(71)
    pairs = _pairs(rng)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("ring", 1)
    engine.set_option("f2w", 3)
    for prm in (engine.Params(), engine.Params(2, -3, 4, 4), engine.Params(1, 0, 0, 0)):
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        for blocks, rows in ((0, 4096), (1, 512), (2, 512), (3, 1024), (7, 512)):
            engine.set_option("blocks", blocks)
            engine.set_option("ring_rows", rows)
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, prm))
                st = engine.last_stats()
                strips = 1 if len(a) <= 192 else (len(a) - 3 + 188) // 189
                if strips > 4:   # more than one group: ring mode on the three-column kernel
                    assert st["variant"] & 8192 and st["variant"] & 4 and st["variant"] & 64 and st["C"] == 64, st
                    assert st["items"] == (strips + 3) // 4, st
            assert got == exp, (prm, blocks, rows)


def test_w3_matches_w2(engine):
    """A 2^17 pair and a 400000 x 400000 pair over 1..4 workgroups per CU (rounds change while a
    ring's consumer still reads the last rows): three columns per lane give the two-column
    kernel's scores."""
    for N, wgs in ((1 << 17, 0), (400000, 1), (400000, 4)):
        a, b = engine.gen_pair(N, N)
        engine.set_option("f2_wgs", wgs)
        engine.set_option("f2w", 2)
        engine.set_option("ring", 1)
        w2 = engine.score(a, b)
        assert engine.last_stats()["variant"] & 16 and not engine.last_stats()["variant"] & 8192
        engine.set_option("f2w", 3)
        w3 = engine.score(a, b)
        st = engine.last_stats()
        assert st["variant"] & 8192 and st["variant"] & 4, st
        assert w3 == w2 > 0, (N, wgs, w3, w2)


def test_w3_config_c5(engine, golden):
    """C5 (N = 2^20, seed 1048576) at three columns per lane against the reference-pinned golden."""
    import torch
    c = golden("configs.json")["C5"]
    N = c["N"]
    a, b = engine.gen_pair(c["seed"], N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.set_option("f2w", 3)
    engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s.cuda_stream)
    engine.stream_status(s.cuda_stream)
    st = engine.last_stats()
    assert st["variant"] & 8192 and st["variant"] & 4 and st["boundary_bytes"] < 1 << 30, st
    assert st["items"] == ((N - 3 + 188) // 189 + 3) // 4, st
    assert score.item() == c["score"]


@pytest.mark.parametrize("nslabs", [2, 3])
def test_w3_slabs(engine, oracle_mod, nslabs):
    """Column slabs on the three-column slab kernel (sw_flow3r3s_kernel): bounds are multiples of
    189 columns, 512-row rings over 3 blocks per slab; max over the slabs = the pair's score."""
    rng = np.random.default_rng(73 + nslabs)
    engine.set_option("f2w", 3)
    engine.set_option("ring_rows", 512)
    engine.set_option("blocks", 3)
    op = oracle_mod.Params(1, -1, 1, 1)
    for n, m in ((nslabs * 2000 + 77, 1500), (nslabs * 1800, 2100)):
        a = _rand_dna(rng, n)
        b = _similar(rng, a, m) if m < n else _rand_dna(rng, m)
        exp = oracle_mod.score_linear(a, b, op)
        got, bounds, stats = _run_threads(engine, a, b, nslabs, engine.SW_FLAG_DNA)
        assert max(got) == exp, (n, m, got, exp, bounds)
        assert all(x % 189 == 0 for x in bounds[1:-1]), bounds
        for s in stats:
            assert s["mode"] == 5 and s["variant"] & 8192 and s["variant"] & 2048, s


# ---- the affine step at three columns per lane (sw_flow3ra3_kernel / sw_flow3ra3s_kernel,
# tools/gen_flow3.py step_aff3): G_INIT != G_EXT, or the affine step forced at G_INIT == G_EXT

AFFINE_SETS = ((2, -3, 5, 2), (1, -1, 3, 1), (1, -1, 1, 3))


def test_w3_affine_ring_parity(engine, oracle_mod):
    rng = np.random.default_rng(75)
    pairs = _pairs(rng)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("ring", 1)
    for prm in AFFINE_SETS + ((1, -1, 2, 2),):
        p = engine.Params(*prm)
        op = oracle_mod.Params(*prm)
        engine.set_option("linear", 0 if prm[2] == prm[3] else -1)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        for blocks, rows in ((0, 4096), (1, 512), (3, 1024), (7, 512)):
            engine.set_option("blocks", blocks)
            engine.set_option("ring_rows", rows)
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, p))
                st = engine.last_stats()
                strips = 1 if len(a) <= 192 else (len(a) - 3 + 188) // 189
                if strips > 4:
                    assert st["variant"] & 8192 and st["variant"] & 1024 and st["variant"] & 4, st
            assert got == exp, (prm, blocks, rows)


def test_w3_affine_matches_w2(engine):
    """A 2^17 pair at (2, -3, 5, 2): three columns per lane give the two-column kernel's score."""
    a, b = engine.gen_pair(1 << 17, 1 << 17)
    p = engine.Params(*AFFINE_SETS[0])
    engine.set_option("ring", 1)
    engine.set_option("f2w", 2)
    w2 = engine.score(a, b, p)
    assert engine.last_stats()["variant"] & 1024 and not engine.last_stats()["variant"] & 8192
    engine.set_option("f2w", 3)
    w3 = engine.score(a, b, p)
    assert engine.last_stats()["variant"] & 8192 and engine.last_stats()["variant"] & 1024
    assert w3 == w2 > 0


@pytest.mark.parametrize("nslabs", [2, 3])
def test_w3_affine_slabs(engine, oracle_mod, nslabs):
    rng = np.random.default_rng(77 + nslabs)
    engine.set_option("ring_rows", 512)
    engine.set_option("blocks", 3)
    prm = AFFINE_SETS[0]
    engine.set_params(engine.Params(*prm))
    op = oracle_mod.Params(*prm)
    for n, m in ((nslabs * 2000 + 77, 1500), (nslabs * 1800, 2100)):
        a = _rand_dna(rng, n)
        b = _similar(rng, a, m) if m < n else _rand_dna(rng, m)
        exp = oracle_mod.score_linear(a, b, op)
        got, bounds, stats = _run_threads(engine, a, b, nslabs, engine.SW_FLAG_DNA)
        assert max(got) == exp, (n, m, got, exp, bounds)
        assert all(x % 189 == 0 for x in bounds[1:-1]), bounds
        for s in stats:
            assert s["variant"] & 8192 and s["variant"] & 1024 and s["variant"] & 2048, s


def test_f3slab_off_keeps_flow2_slab_kernel(engine, oracle_mod):
    """Option f3slab = 0 keeps a ring-mode column slab on flow2's slab kernel (no three-column form):
    slab bounds on its strip stride (not 189), the slabs score the pair, and the same cut with
    f3slab = 1 runs flow3's three-column slab kernel to the same maximum."""
    rng = np.random.default_rng(81)
    a = _rand_dna(rng, 2 * 2000 + 77)
    b = _similar(rng, a, 1500)
    exp = oracle_mod.score_linear(a, b, oracle_mod.Params(1, -1, 1, 1))
    engine.set_option("ring", 1)
    engine.set_option("ring_rows", 512)
    engine.set_option("blocks", 3)
    try:
        engine.set_option("f3slab", 0)
        q0 = engine.slab_bounds(len(a), len(b), 2, engine.SW_FLAG_DNA)
        got, bounds, stats = _run_threads(engine, a, b, 2, engine.SW_FLAG_DNA)
        assert bounds == q0 and max(got) == exp, (got, exp, bounds)
        for st in stats:
            assert st["mode"] == 5 and st["variant"] & 4 and not st["variant"] & (2048 | 8192), st
        assert bounds[1] % 63 == 0, bounds   # flow2's strip stride (63 or 126 columns)
        engine.set_option("f3slab", 1)
        got1, bounds1, stats1 = _run_threads(engine, a, b, 2, engine.SW_FLAG_DNA)
        assert max(got1) == exp and bounds1[1] % 189 == 0, (got1, bounds1)
        for st in stats1:
            assert st["variant"] & 2048 and st["variant"] & 8192, st
    finally:
        engine.set_option("f3slab", 1)
