"""GPU parity: flow2 with two columns per lane (option f2w = 2, sw_flow2.hip W2:
strips of 128 columns overlapping by two, the linear-gap step) against the oracle,
bit-exact.  Ragged shapes around the 126-column stride and the 4-strip groups, the
staged kernel with its loader wave on small grids, streamed row codes, ring edges,
column slabs, and the C2 pair at full size."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)
OPTS = ("W", "C", "blocks", "orient", "f2stream", "f2_wgs")


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
        for k in OPTS:
            engine.set_option(k, 0)
        engine.set_option("mode", -1)
        engine.set_option("ring", -1)
        engine.set_option("ring_rows", 4096)
        engine.set_option("linear", -1)
        engine.set_option("f2w", 0)
    reset()
    yield
    reset()


SHAPES = [(1, 1), (1, 200), (200, 1), (2, 5), (63, 63), (64, 64), (126, 127), (127, 126), (128, 300), (129, 129),
          (130, 64), (252, 253), (253, 252), (254, 255), (255, 1000), (256, 17), (505, 505), (1000, 64), (2017, 2100),
          (4096, 4000), (5041, 777)]


def test_w2_ragged(engine, oracle_mod):
    """Ragged shapes, C = 32 and 64, one-workgroup and automatic grids, several
    pairs per launch, three linear-gap constant sets."""
    rng = np.random.default_rng(7)
    pairs = _pairs(rng, SHAPES)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("f2w", 2)
    for prm in (engine.Params(), engine.Params(2, -3, 4, 4), engine.Params(1, 0, 0, 0)):
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        for C in (32, 64):
            engine.set_option("C", C)
            got = [engine.score(a, b, prm) for a, b in pairs]
            assert got == exp, (prm, C)
            st = engine.last_stats()
            assert st["mode"] == 5 and st["variant"] & 16 and st["variant"] & 8, st
            assert engine.score_batch(pairs, prm) == exp, (prm, C)
            for blocks in (1, 3):
                engine.set_option("blocks", blocks)
                assert engine.score_batch(pairs, prm) == exp, (prm, C, blocks)
            engine.set_option("blocks", 0)


def test_w2_needs_the_linear_step(engine, oracle_mod):
    """G_INIT != G_EXT, or the affine step forced (linear = 0): W = 1 runs instead."""
    rng = np.random.default_rng(8)
    a, b = _pairs(rng, [(2017, 2100)])[0]
    engine.set_option("mode", 5)
    engine.set_option("f2w", 2)
    prm = engine.Params(2, -3, 5, 2)
    assert engine.score(a, b, prm) == oracle_mod.score_linear(a, b, oracle_mod.Params(2, -3, 5, 2))
    assert not engine.last_stats()["variant"] & 16
    engine.set_option("linear", 0)
    assert engine.score(a, b) == oracle_mod.score_linear(a, b)
    assert not engine.last_stats()["variant"] & 16


def test_w2_streamed_and_ring(engine, oracle_mod):
    """Streamed row codes, and ring edges on grids of 1, 2, 3 and 7 blocks with
    512-row rings (many rounds, the wrap ring every round)."""
    rng = np.random.default_rng(9)
    pairs = _pairs(rng, [(253, 700), (1009, 513), (2017, 3001), (4096, 2600), (5000, 1200), (9000, 2000)])
    exp = [oracle_mod.score_linear(a, b) for a, b in pairs]
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("f2w", 2)
    engine.set_option("f2stream", 1)
    for C in (32, 64):
        engine.set_option("C", C)
        assert [engine.score(a, b) for a, b in pairs] == exp, C
        assert engine.last_stats()["variant"] & 18 == 18
    engine.set_option("C", 0)
    engine.set_option("f2stream", 0)
    engine.set_option("ring", 1)
    for blocks, rows in ((0, 4096), (1, 512), (2, 512), (3, 1024), (7, 512)):
        engine.set_option("blocks", blocks)
        engine.set_option("ring_rows", rows)
        got = []
        for a, b in pairs:
            got.append(engine.score(a, b))
            st = engine.last_stats()
            groups = (((len(a) - 2 + 125) // 126 if len(a) > 128 else 1) + 3) // 4
            assert st["variant"] & 16 and bool(st["variant"] & 4) == (groups > 1), st
        assert got == exp, (blocks, rows)


def test_w2_slab_bounds_are_126_column_multiples(engine):
    engine.set_option("f2w", 2)
    b = engine.slab_bounds(100000, 5000, 3, engine.SW_FLAG_DNA)
    assert b[0] == 0 and b[-1] == 100000
    assert all(x % 126 == 0 for x in b[:-1]), b
    engine.set_option("f2w", 1)
    b1 = engine.slab_bounds(100000, 5000, 3, engine.SW_FLAG_DNA)
    assert all(x % 63 == 0 for x in b1[:-1]) and b1 != b, b1


def test_w2_config_c2(engine, golden):
    """C2 (N = 65536, seed 65536) with two columns per lane against its golden."""
    import torch
    c = golden("configs.json")["C2"]
    N = c["N"]
    a, b = engine.gen_pair(c["seed"], N)
    engine.set_option("f2w", 2)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s.cuda_stream)
    engine.stream_status(s.cuda_stream)
    st = engine.last_stats()
    assert st["mode"] == 5 and st["variant"] & 16 and not st["variant"] & 2, st
    assert score.item() == c["score"]
