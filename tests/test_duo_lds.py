"""GPU parity of the duo kernel with every strip hand-off in LDS (sw_kernels.hip
sw_duo_lds_kernel, option duo_lds, variant bit 128) against the oracle and against the
granule duo kernel (duo_lds = 0) on the same inputs.  Bit-exact integer equality.

Covered: strips per duo 1..7 (rounds with idle waves), rows around the 64-row chunk and
the 511-step lane skew, ragged pairs padded inside a duo, the linear-gap and the affine
step (4- and 8-byte slots), grids of 1-3 workgroups (many duos per workgroup, rounds
crossing duos), the row codes from the LDS table (duo_tab = 1, W = 4 / 8) and carried by DPP
(duo_tab = 0), rows beyond the table's or the wrap buffer's LDS (the next kernel down then), and
C3 in full against its golden."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _rand_dna(rng, n):
    return ACGT[rng.integers(0, 4, n)]


def _related(rng, n, m, p=0.1):
    a = _rand_dna(rng, n)
    b = np.resize(a, m).copy()
    mut = rng.random(m) < p
    b[mut] = _rand_dna(rng, int(mut.sum()))
    return a, b


@pytest.fixture(autouse=True)
def _defaults(engine):
    yield
    for k in ("blocks", "W", "C"):
        engine.set_option(k, 0)
    engine.set_option("mode", -1)
    engine.set_option("duo_lds", 1)
    engine.set_option("duo_tab", 1)
    engine.set_option("linear", -1)


def _check(engine, oracle_mod, pairs, prm, lds_expected=True, W=8, tab_expected=None):
    """The duo kernel at W columns per lane and 64-row chunks (the LDS links' chunk)."""
    op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
    exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
    engine.set_option("mode", 3)
    engine.set_option("W", W)
    engine.set_option("C", 64)
    engine.set_option("duo_lds", 1)
    got = engine.score_batch(pairs, prm)
    st = engine.last_stats()
    assert st["mode"] == 3 and st["W"] == W and st["C"] == 64, st
    assert bool(st["variant"] & 128) == lds_expected, st
    if lds_expected:
        assert st["boundary_bytes"] == 0, st
    if tab_expected is not None:
        assert bool(st["variant"] & 256) == tab_expected, st
    assert got == exp, ("lds", prm)
    engine.set_option("duo_lds", 0)
    assert engine.score_batch(pairs, prm) == exp, ("granules", prm)
    assert not engine.last_stats()["variant"] & 128
    engine.set_option("duo_lds", 1)
    return exp


PARAMS = [(1, -1, 1, 1), (2, -3, 5, 2), (3, -1, 4, 1), (3, -2, 5, 5)]


@pytest.mark.parametrize("prm_t", PARAMS)
def test_duo_lds_strip_counts_and_rows(engine, oracle_mod, prm_t):
    """Duos of 1..7 strips (W = 8: 512 columns each, W = 4: 256; rounds with 1-3 idle waves) and rows
    around the chunk and the lane skew, as ragged pairs; the linear-gap and affine steps."""
    prm = engine.Params(*prm_t)
    rng = np.random.default_rng(1000 + sum(prm_t))
    ns = [100, 512, 513, 1100, 1600, 2048, 2100, 2700, 3500]
    ms = [1, 2, 63, 64, 65, 511, 512, 513, 575, 1000, 2049]
    pairs = []
    for i in range(14):
        n, m = ns[i % len(ns)], ms[(3 * i) % len(ms)]
        pairs.append(_related(rng, n, m) if i % 3 else (_rand_dna(rng, n), _rand_dna(rng, m)))
    for lin in ((-1, 0) if prm.gap_init == prm.gap_ext else (-1,)):
        engine.set_option("linear", lin)
        for W in (8, 4):
            for tab in (1, 0):
                engine.set_option("duo_tab", tab)
                _check(engine, oracle_mod, pairs, prm, W=W, tab_expected=bool(tab))
        engine.set_option("duo_tab", 1)


def test_duo_lds_grids_many_duos(engine, oracle_mod):
    """11 duos on grids of 1, 2 and 3 workgroups: a workgroup's waves run from one duo into the
    next (positions continuing across rounds and duos; with the code table, wave 0 rewrites it
    for the next duo once every wave is done with the last), table and DPP codes."""
    rng = np.random.default_rng(9)
    pairs = [_related(rng, int(rng.integers(300, 4200)), int(rng.integers(50, 3000))) for _ in range(22)]
    for prm in (engine.Params(), engine.Params(2, -3, 5, 2)):
        for tab in (1, 0):
            engine.set_option("duo_tab", tab)
            for blocks in (1, 2, 3):
                engine.set_option("blocks", blocks)
                _check(engine, oracle_mod, pairs, prm, tab_expected=bool(tab))
    engine.set_option("blocks", 0)
    engine.set_option("duo_tab", 1)


def test_duo_lds_wrap_buffer_limit(engine, oracle_mod):
    """The LDS kernel's dynamic LDS admits two workgroups per CU: with the code table up to
    m_pad = 8192 at the linear-gap step (4-B slots: 32 KB wrap buffer + 38 KB table) and 4096
    affine; without the table the wrap buffer alone up to 16384 / 8192; longer rows take the
    granule kernel.  Same scores everywhere."""
    rng = np.random.default_rng(4)
    for lin, cases in ((True, ((8192, True, True), (8193, True, False), (16384, True, False), (16385, False, False))),
                       (False, ((4096, True, True), (4097, True, False), (8192, True, False), (8193, False, False)))):
        p = engine.Params() if lin else engine.Params(2, -3, 5, 2)
        for m, lds, tab in cases:
            pairs = [_related(rng, 700, m), _related(rng, 1300, m - 7), (_rand_dna(rng, 90), _rand_dna(rng, 40))]
            _check(engine, oracle_mod, pairs, p, lds_expected=lds, tab_expected=tab if lds else None)


def test_duo_lds_c3_golden(engine, golden):
    """C3 (1024 pairs N = 8192, the reference-pinned golden) on the LDS duo kernel, row codes
    from the LDS table and by DPP, strip roles per CU and by wave index; no strip-boundary
    buffer in HBM."""
    c = golden("configs.json")["C3"]
    N = c["N"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], N)
    pairs = [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]
    try:
        for tab, roles in ((1, 1), (1, 0), (0, 1)):
            engine.set_option("duo_tab", tab)
            engine.set_option("duo_roles", roles)
            got = engine.score_batch(pairs)
            st = engine.last_stats()
            assert st["mode"] == 3 and st["variant"] & 128 and st["boundary_bytes"] == 0, st
            assert bool(st["variant"] & 256) == bool(tab), st
            assert got == c["scores"], (tab, roles)
    finally:
        engine.set_option("duo_roles", 1)


def test_duo_lds_priority_turns(engine, golden):
    """Turn-taking at issue priority between a CU's two workgroups (option duo_prio: -1 auto = 1.3 ms
    slices on the LDS-table kernel, 0 off, short and long slices) changes timing only: C3 scores
    equal the golden under each; out-of-range values are refused."""
    c = golden("configs.json")["C3"]
    N = c["N"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], N)
    pairs = [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]
    try:
        for k in (-1, 0, 6, 17):
            engine.set_option("duo_prio", k)
            assert engine.get_option("duo_prio") == k
            assert engine.score_batch(pairs) == c["scores"], k
            assert engine.last_stats()["variant"] & 256
        for bad in (-2, 1, 5, 21):
            with pytest.raises(engine.SwError):
                engine.set_option("duo_prio", bad)
    finally:
        engine.set_option("duo_prio", -1)


def test_duo_lds_table_multi_pass_long_rows(engine, oracle_mod):
    """Batches of more duos than two per CU take the LDS-table kernel when their rows reach 8192 (the
    table is rewritten per duo, workgroups taking turns at priority): 1100 pairs of 8192 rows x 64..320
    columns, against the table-less kernel (duo_tab = 0) and the oracle on a sample."""
    rng = np.random.default_rng(21)
    pairs = []
    for k in range(1100):
        n = int(rng.integers(64, 321))
        pairs.append(_related(rng, n, 8192) if k % 2 else (_rand_dna(rng, n), _rand_dna(rng, 8192)))
    engine.set_option("orient", 1)
    engine.set_option("mode", 3)
    engine.set_option("W", 8)
    engine.set_option("C", 64)
    try:
        engine.set_option("duo_tab", 1)
        tab = engine.score_batch(pairs)
        st = engine.last_stats()
        assert st["mode"] == 3 and st["variant"] & 128 and st["variant"] & 256 and st["items"] == 550, st
        engine.set_option("duo_tab", 0)
        plain = engine.score_batch(pairs)
        assert not engine.last_stats()["variant"] & 256
        assert tab == plain
        op = oracle_mod.Params(1, -1, 1, 1)
        for k in range(0, 1100, 157):
            assert tab[k] == oracle_mod.score_linear(pairs[k][0], pairs[k][1], op), k
    finally:
        engine.set_option("orient", 0)
