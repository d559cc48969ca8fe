"""GPU parity: the flow3 kernel (sw_flow3.hip: flow2's staged two-column linear-gap
kernel with hand-scheduled chunk loops, tools/gen_flow3.py) against the oracle,
bit-exact, and against flow2 (option f3 = 0) on the same inputs.  Ragged shapes
around the 126-column strip stride, the 4-strip groups and the 64-row chunk pairs,
every strip role (no inflow / LDS inflow x no outflow / LDS / granules), grids of
1-3 workgroups (groups run in rounds through the loader's granule path), several
pairs per launch, three linear-gap constant sets and C2 in full."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _rand_dna(rng, n):
    return ACGT[rng.integers(0, 4, n)]


def _pairs(rng, shapes):
    out = []
    for n, m in shapes:
        a = _rand_dna(rng, n)
        b = _rand_dna(rng, m)
        if rng.random() < 0.5 and m > 10:
            b = np.resize(a, m).copy()        # long diagonals through every strip edge
            mut = rng.random(m) < 0.05
            b[mut] = _rand_dna(rng, int(mut.sum()))
        out.append((a, b))
    return out


@pytest.fixture(autouse=True)
def _defaults(engine):
    def reset():
        engine.set_params(engine.Params())
        for k in ("W", "C", "blocks", "orient", "f2w"):
            engine.set_option(k, 0)
        engine.set_option("mode", -1)
        engine.set_option("linear", -1)
        engine.set_option("f3", 1)
        engine.set_option("f3hl", 1)
    reset()
    yield
    reset()


# rows around the 64-row chunk pairs and the ring's 512 rows, columns around the
# 126-column strips and 504-column groups (1, 2, 4, 5, 8, 9 strips)
SHAPES = [(1, 1), (1, 200), (200, 1), (2, 5), (126, 127), (128, 63), (129, 64), (130, 65), (252, 95), (253, 96),
          (254, 97), (505, 505), (506, 511), (1000, 512), (1008, 513), (1009, 1000), (1135, 1100), (2017, 2100),
          (4096, 4000), (5041, 777)]


def test_flow3_ragged(engine, oracle_mod):
    rng = np.random.default_rng(31)
    pairs = _pairs(rng, SHAPES)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)      # flow2 planning for every shape (single strips included)
    engine.set_option("f2w", 2)
    for C, hl in ((32, 0), (16, 0), (32, 1)):   # 32- and 16-row chunks; 32 with half-chunk LDS links
        engine.set_option("C", C)
        engine.set_option("f3hl", hl)
        for prm in (engine.Params(), engine.Params(2, -3, 4, 4), engine.Params(1, 0, 0, 0)):
            op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, prm))
                st = engine.last_stats()
                assert st["mode"] == 5 and st["variant"] & 64 and st["variant"] & 16 and st["C"] == C, st
                assert bool(st["variant"] & 512) == bool(hl), st
            assert got == exp, (prm, C)
            assert engine.score_batch(pairs, prm) == exp, (prm, C)
            for blocks in (1, 2, 3):
                engine.set_option("blocks", blocks)
                assert engine.score_batch(pairs, prm) == exp, (prm, blocks, C)
            engine.set_option("blocks", 0)
    engine.set_option("C", 0)


def test_flow3_matches_flow2(engine):
    """The same launches on flow2 (option f3 = 0) give the same scores."""
    rng = np.random.default_rng(32)
    pairs = _pairs(rng, [(3001, 2999), (6000, 1500), (1500, 6000), (777, 9000)])
    engine.set_option("mode", 5)      # a batch on the staged flow2 plan (not the streamed item claim)
    engine.set_option("W", 1)
    got3 = engine.score_batch(pairs)
    assert engine.last_stats()["variant"] & 64
    engine.set_option("f3", 0)
    got2 = engine.score_batch(pairs)
    assert not engine.last_stats()["variant"] & 64
    assert got3 == got2


def test_flow3_only_where_it_applies(engine, oracle_mod):
    """The affine step (G_INIT != G_EXT, or linear = 0) runs flow3's affine kernel (variant bit
    1024, test_flow3_affine.py), not the two-column one; C = 64 stays on flow2."""
    rng = np.random.default_rng(33)
    a, b = _pairs(rng, [(2017, 2100)])[0]
    prm = engine.Params(2, -3, 5, 2)
    assert engine.score(a, b, prm) == oracle_mod.score_linear(a, b, oracle_mod.Params(2, -3, 5, 2))
    assert not engine.last_stats()["variant"] & 64 and engine.last_stats()["variant"] & 1024
    engine.set_option("linear", 0)
    assert engine.score(a, b) == oracle_mod.score_linear(a, b)
    assert not engine.last_stats()["variant"] & 64 and engine.last_stats()["variant"] & 1024
    engine.set_option("linear", -1)
    engine.set_option("C", 64)
    engine.set_option("mode", 5)
    assert engine.score(a, b) == oracle_mod.score_linear(a, b)
    assert not engine.last_stats()["variant"] & 64


def test_flow3_config_c2(engine, golden):
    """C2 (N = 65536, seed 65536) on flow3 against its golden."""
    import torch
    c = golden("configs.json")["C2"]
    N = c["N"]
    a, b = engine.gen_pair(c["seed"], N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    try:
        for hl in (1, 0, 1):   # the default (32-row chunks, half-chunk LDS links), then 16-row chunks
            engine.set_option("f3hl", hl)
            engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1,
                                      stream=s.cuda_stream)
            engine.stream_status(s.cuda_stream)
            st = engine.last_stats()
            assert st["mode"] == 5 and st["variant"] & 64 and not st["variant"] & 2, st
            assert bool(st["variant"] & 512) == bool(hl) and st["C"] == (32 if hl else 16), st
            assert score.item() == c["score"]
    finally:
        engine.set_option("f3hl", 1)


# ---- ring mode (sw_flow3.hip sw_flow3r_kernel: streamed row codes, group edges through
# per-block rings, C = 64 or 32; the C5 organisation)

def _ring_opts(engine, blocks, rows):
    engine.set_option("ring", 1)
    engine.set_option("blocks", blocks)
    engine.set_option("ring_rows", rows)


@pytest.fixture
def _ring_reset(engine):
    yield
    engine.set_option("ring", -1)
    engine.set_option("ring_rows", 4096)
    engine.set_option("blocks", 0)
    engine.set_option("f3rhl", 0)


def test_flow3_ring_parity(engine, oracle_mod, _ring_reset):
    """Ring mode forced on grids of 1, 2, 3 and 7 blocks with 512-row rings (many rounds,
    the wrap ring every round), rows around the 64-row chunk pairs, three constant sets."""
    rng = np.random.default_rng(34)
    pairs = _pairs(rng, [(253, 700), (1009, 513), (2017, 3001), (4096, 2600), (5000, 1200), (9000, 2000),
                         (3025, 127), (2521, 129)])
    engine.set_option("orient", 1)
    for prm in (engine.Params(), engine.Params(2, -3, 4, 4), engine.Params(1, 0, 0, 0)):
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        # 64-row chunks (automatic in ring mode) at two columns per lane (option f2w = 2) and at
        # three (automatic, tests/test_ring_w3.py), 32 (option C), 64 with half-chunk LDS links
        for C, hl, f2w in ((64, 0, 2), (64, 0, 0), (32, 0, 0), (64, 1, 0)):
            engine.set_option("C", 0 if C == 64 else C)
            engine.set_option("f3rhl", hl)
            engine.set_option("f2w", f2w)
            w3 = C == 64 and not hl and f2w == 0
            for blocks, rows in ((0, 4096), (1, 512), (2, 512), (3, 1024), (7, 512)):
                _ring_opts(engine, blocks, rows)
                got = []
                for a, b in pairs:
                    got.append(engine.score(a, b, prm))
                    st = engine.last_stats()
                    groups = (((len(a) - 2 + 125) // 126 if len(a) > 128 else 1) + 3) // 4
                    if groups > 1:
                        assert st["variant"] & 64 and st["variant"] & 4 and st["C"] == C, st
                        assert bool(st["variant"] & 512) == bool(hl), st
                        assert bool(st["variant"] & 8192) == w3, st
                assert got == exp, (prm, C, f2w, blocks, rows)
        engine.set_option("C", 0)
        engine.set_option("f2w", 0)


def test_flow3_ring_matches_flow2(engine, _ring_reset):
    """A 2^17 pair in ring mode (520 groups) on flow3 and on flow2 (f3 = 0): the same score."""
    import torch
    N = 1 << 17
    a, b = engine.gen_pair(N, N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.set_option("ring", 1)
    out = []
    try:
        for f3, C, hl in ((1, 0, 0), (1, 32, 0), (1, 0, 1), (0, 0, 0)):
            engine.set_option("f3", f3)
            engine.set_option("C", C)
            engine.set_option("f3rhl", hl)
            engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1,
                                      stream=s.cuda_stream)
            engine.stream_status(s.cuda_stream)
            st = engine.last_stats()
            assert bool(st["variant"] & 64) == bool(f3) and st["variant"] & 4 and st["C"] == (C or 64), st
            out.append(score.item())
    finally:
        engine.set_option("f3", 1)
        engine.set_option("C", 0)
    assert out[0] == out[1] == out[2] == out[3] > 0
