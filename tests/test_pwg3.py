"""GPU parity: batches whose scores need int32 on flow3's three-column ring step with a pair per
workgroup (sw_flow3.hip sw_flow3r3p_kernel, sw_engine.hip plan_pwg3): each workgroup runs its pairs'
strip groups one after another, wave 3 handing each group's edge to the next group's wave 0 through the
workgroup's own ring of 8-B granules.  The linear-gap step (main.cpp:54-66 at G_INIT == G_EXT, exact,
DESIGN.md section 2), bit-exact against the oracle (lazySmith.cpp:15-69 restated), against flow2's
pair-per-workgroup kernel (option f3pwg = 0) and against the C3 golden."""
import numpy as np
import pytest

from test_slab import _rand_dna, _similar

pytestmark = pytest.mark.gpu

PWG3 = 32768   # variant bit of sw_flow3r3p_kernel


@pytest.fixture(autouse=True)
def _defaults(engine):
    def reset():
        engine.set_params(engine.Params())
        for k in ("W", "C", "blocks", "orient"):
            engine.set_option(k, 0)
        engine.set_option("mode", -1)
        engine.set_option("f2pwg", -1)
        engine.set_option("f3pwg", 1)
        engine.set_option("linear", -1)
    reset()
    yield
    reset()


def _forced(engine):
    engine.set_option("mode", 5)
    engine.set_option("f2pwg", 1)


def test_pwg3_ragged_parity(engine, oracle_mod):
    """Ragged pairs around the 189-column strips, the 756-column groups and the 64-row chunks (one to
    nine groups per pair, rows 1..3000), on grids of 1, 3 and 7 workgroups (workgroups running several
    pairs in turn) and the automatic grid; three linear-gap constant sets and three affine ones
    (G_INIT > G_EXT, G_INIT < G_EXT) on the affine ring step."""
    rng = np.random.default_rng(33)
    shapes = [(1, 1), (5, 300), (192, 64), (193, 65), (380, 129), (756, 700), (757, 1000), (1513, 63),
              (2000, 2049), (3000, 511), (4000, 1500), (6805, 3000), (300, 1)]
    pairs = []
    for n, m in shapes:
        a = _rand_dna(rng, n)
        pairs.append((a, _similar(rng, a, m)) if m > 10 and rng.random() < 0.6 else (a, _rand_dna(rng, m)))
    engine.set_option("orient", 1)
    _forced(engine)
    for prm in ((1, -1, 1, 1), (2, -3, 2, 2), (3, 0, 4, 4), (2, -3, 5, 2), (1, -1, 3, 1), (1, -1, 1, 3)):
        p = engine.Params(*prm)
        exp = [oracle_mod.score_linear(a, b, oracle_mod.Params(*prm)) for a, b in pairs]
        for blocks in (1, 3, 7, 0):
            engine.set_option("blocks", blocks)
            got = engine.score_batch(pairs, p)
            st = engine.last_stats()
            lin = prm[2] == prm[3]
            # the linear-gap ring step (variant 8) or the affine one (1024: sw_flow3ra3p_kernel)
            assert st["mode"] == 5 and st["variant"] & PWG3, (prm, blocks, st)
            assert bool(st["variant"] & 8) == lin and bool(st["variant"] & 1024) == (not lin), (prm, st)
            assert got == exp, (prm, blocks, [(k, got[k], exp[k]) for k in range(len(exp)) if got[k] != exp[k]][:5])


def test_pwg3_matches_flow2_pwg_c3(engine, golden):
    """C3 (1024 pairs N = 8192) forced onto the int32 kernels: flow3's three-column pair-per-workgroup
    kernel and flow2's (f3pwg = 0) both give the reference-pinned golden."""
    c = golden("configs.json")["C3"]
    N = c["N"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], N)
    pairs = [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]
    _forced(engine)
    assert engine.score_batch(pairs) == c["scores"]
    st = engine.last_stats()
    assert st["variant"] & PWG3 and st["items"] == 1024, st
    engine.set_option("f3pwg", 0)
    assert engine.score_batch(pairs) == c["scores"]
    assert not engine.last_stats()["variant"] & PWG3


def test_pwg3_automatic_int32_batch(engine, oracle_mod):
    """A batch whose scores pass 2^16 (similar pairs of 20000 at MATCH = 4: no 16-bit duos) takes the
    three-column pair-per-workgroup kernel on the automatic plan; scores against the oracle on a sample
    and against flow2's kernel in full."""
    rng = np.random.default_rng(34)
    pairs = []
    for k in range(600):
        n = int(rng.integers(17000, 20001))
        a = _rand_dna(rng, n)
        pairs.append((a, _similar(rng, a, int(rng.integers(16000, 20001)))))
    p = engine.Params(4, -3, 2, 2)
    got = engine.score_batch(pairs, p)
    st = engine.last_stats()
    assert st["mode"] == 5 and st["variant"] & PWG3, st
    assert max(got) >= 1 << 16, max(got)
    op = oracle_mod.Params(4, -3, 2, 2)
    for k in (0, 299, 599):
        assert got[k] == oracle_mod.score_linear(pairs[k][0], pairs[k][1], op), k
    engine.set_option("f3pwg", 0)
    assert engine.score_batch(pairs, p) == got
    assert not engine.last_stats()["variant"] & PWG3


def test_pwg3_affine_c3_golden(engine, golden):
    """C3 at (2, -3, 5, 2) forced onto the int32 kernels (its scores fit 16 bits): flow3's three-column
    affine pair-per-workgroup kernel and flow2's one-column one both give C3_affine (the reference's
    refvar LazySmith)."""
    c = golden("configs.json")["C3_affine"]
    N = c["N"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], N)
    pairs = [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]
    p = engine.Params(*c["params"])
    _forced(engine)
    assert engine.score_batch(pairs, p) == c["scores"]
    st = engine.last_stats()
    assert st["variant"] & PWG3 and st["variant"] & 1024 and not st["variant"] & 8, st
    engine.set_option("f3pwg", 0)
    assert engine.score_batch(pairs, p) == c["scores"]
    assert not engine.last_stats()["variant"] & PWG3
