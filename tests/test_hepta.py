"""GPU parity of single pairs over alphabets of up to seven byte values other than {A,C,G,T}
(ACGTN, lower-case acgt, RNA, any seven bytes) on flow3's staged kernels (sw_flow3.hip HEP:
3-bit row symbols, the perms' low source word per column; sw_engine.hip set_hep /
hep_staged), against the oracle and against the byte path (option hep = 0).  Bit-exact
integer equality.  main.cpp:28-33 scores by byte equality, so a pair's byte values are its
alphabet.

Covered: alphabets of 1..7 values (0x00 and 0xFF among them), the linear-gap (two columns per
lane) and affine (one column) staged kernels at C = 32 with half-chunk links and at C = 16,
ragged strips, the host entry points and the device entry point (the alphabet kernel's byte
set); the three-column ring kernels (rows too long for LDS, or option ring = 1) over rows translated
to selectors; fallbacks to the byte path: eight values, option hep = 0, the pool loops; C2- and
C5-size ACGTN pairs against the byte path."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ALPHABETS = {
    "acgtn": b"ACGTN",
    "lower": b"acgt",
    "rna": b"ACGU",
    "seven": bytes([0x00, 0x41, 0x7F, 0x80, 0xFE, 0xFF, 0x2D]),
    "two": b"XY",
    "one": b"Q",
}
HEP_BIT = 65536


def _rand(rng, alpha, n):
    a = np.frombuffer(alpha, np.uint8)
    return a[rng.integers(0, len(a), n)]


def _related(rng, alpha, n, m, p=0.15):
    a = _rand(rng, alpha, n)
    b = np.resize(a, m).copy()
    mut = rng.random(m) < p
    b[mut] = _rand(rng, alpha, int(mut.sum()))
    return a, b


@pytest.fixture(autouse=True)
def _defaults(engine):
    yield
    for k, v in (("hep", 1), ("C", 0), ("W", 0), ("f3hl", 1), ("f3pool", 0), ("mode", -1), ("ring", -1), ("f3rhl", 0)):
        engine.set_option(k, v)


def _score(engine, a, b, prm):
    got = engine.score(a, b, prm)
    return got, engine.last_stats()


@pytest.mark.parametrize("alpha", sorted(ALPHABETS))
@pytest.mark.parametrize("prm_t", [(1, -1, 1, 1), (2, -3, 5, 2), (3, -2, 2, 2)])
def test_hepta_pairs(engine, oracle_mod, alpha, prm_t):
    """Ragged single pairs over each alphabet: the staged flow3 kernel with the seven-letter
    profiles (stats dna = 2, variant bit 16), equal to the oracle."""
    rng = np.random.default_rng(zlib.crc32(repr((alpha, prm_t)).encode()))
    prm = engine.Params(*prm_t)
    op = oracle_mod.Params(*prm_t)
    shapes = [(300, 200), (1000, 1000), (2600, 700), (4100, 3000)]
    for k, (n, m) in enumerate(shapes):
        a, b = _related(rng, ALPHABETS[alpha], n, m) if k % 2 else (_rand(rng, ALPHABETS[alpha], n),
                                                                      _rand(rng, ALPHABETS[alpha], m))
        got, st = _score(engine, a, b, prm)
        assert st["dna"] == 2 and st["variant"] & HEP_BIT, (alpha, st)
        assert got == oracle_mod.score_linear(a, b, op), (alpha, prm_t, n, m)


@pytest.mark.parametrize("C,hl", [(32, 1), (32, 0), (16, 0)])
def test_hepta_chunk_forms(engine, oracle_mod, C, hl):
    """C = 32 with and without half-chunk links and C = 16, both steps, an ACGTN pair of
    ~10k with long related runs."""
    rng = np.random.default_rng(C + hl)
    a, b = _related(rng, ALPHABETS["acgtn"], 9000, 7000, 0.05)
    engine.set_option("f3hl", hl)
    engine.set_option("C", C)
    for prm_t in ((1, -1, 1, 1), (2, -3, 5, 2)):
        got, st = _score(engine, a, b, engine.Params(*prm_t))
        assert st["dna"] == 2 and st["C"] == C, st
        assert got == oracle_mod.score_linear(a, b, oracle_mod.Params(*prm_t)), (C, hl, prm_t)


def test_hepta_fallbacks(engine, oracle_mod):
    """Eight byte values, option hep = 0, the pool loops and a ring plan without a seven-letter form keep the
    byte path; all equal."""
    rng = np.random.default_rng(3)
    a, b = _related(rng, b"ACGTacgt", 3000, 2500)
    got, st = _score(engine, a, b, engine.Params())
    assert st["dna"] == 0 and not st["variant"] & HEP_BIT, st
    assert got == oracle_mod.score_linear(a, b, oracle_mod.Params(1, -1, 1, 1))
    a, b = _related(rng, b"ACGTN", 3000, 2500)
    exp = oracle_mod.score_linear(a, b, oracle_mod.Params(1, -1, 1, 1))
    engine.set_option("hep", 0)
    got, st = _score(engine, a, b, engine.Params())
    assert st["dna"] == 0 and got == exp, st
    engine.set_option("hep", 1)
    engine.set_option("f3pool", 1)
    got, st = _score(engine, a, b, engine.Params())
    assert st["dna"] == 0 and got == exp, st
    # a ring plan without the seven-letter form (half-chunk ring links: two columns per lane) re-plans
    # from scratch on the byte path
    engine.set_option("f3pool", 0)
    engine.set_option("ring", 1)
    engine.set_option("f3rhl", 1)
    got, st = _score(engine, a, b, engine.Params())
    assert st["dna"] == 0 and not st["variant"] & 4 and got == exp, st


def test_hepta_device_entry(engine, oracle_mod):
    """The device entry point with no alphabet flag: the alphabet kernel's byte set picks the
    seven-letter path for one pair, and a batch of two keeps the duo byte path."""
    import torch
    rng = np.random.default_rng(8)
    a, b = _related(rng, ALPHABETS["seven"], 5000, 4000)
    exp = oracle_mod.score_linear(a, b, oracle_mod.Params(1, -1, 1, 1))
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    sc = torch.zeros(2, dtype=torch.int32, device="cuda")
    engine.score_batch_device(arena.data_ptr(), [0], [len(a)], [len(a)], [len(b)], sc.data_ptr())
    st = engine.last_stats()
    assert st["dna"] == 2 and sc[0].item() == exp, st
    engine.score_batch_device(arena.data_ptr(), [0, 0], [len(a), len(a)], [len(a), len(a)], [len(b), len(b)],
                              sc.data_ptr())
    assert engine.last_stats()["dna"] == 0 and sc.tolist() == [exp, exp]


def test_hepta_c2_size_acgtn(engine):
    """N = 65536 with 1 % N (C2's shape): the seven-letter path equals the byte path (hep = 0)."""
    rng = np.random.default_rng(65536)
    a, b = engine.gen_pair(65536, 65536)
    a, b = a.copy(), b.copy()
    a[rng.random(65536) < 0.01] = ord("N")
    b[rng.random(65536) < 0.01] = ord("N")
    got = engine.SmithWatermanScoreCUDA(a, b)
    st = engine.last_stats()
    assert st["dna"] == 2 and st["variant"] & HEP_BIT, st
    engine.set_option("hep", 0)
    ref = engine.SmithWatermanScoreCUDA(a, b)
    assert engine.last_stats()["dna"] == 0
    assert got == ref


@pytest.mark.parametrize("prm_t", [(1, -1, 1, 1), (2, -3, 5, 2)])
def test_hepta_ring_mode(engine, oracle_mod, prm_t):
    """Ring mode (option ring = 1 on pairs the oracle scores in seconds): the three-column ring
    kernels over seven-letter rows translated to selectors (sw_flow3r3h / ra3h_kernel), ragged
    shapes, equal to the oracle."""
    rng = np.random.default_rng(17 + prm_t[0])
    op = oracle_mod.Params(*prm_t)
    engine.set_option("ring", 1)
    try:
        for k, (n, m) in enumerate([(5000, 3000), (12000, 9000), (800, 20000)]):
            alpha = (ALPHABETS["acgtn"], ALPHABETS["seven"], ALPHABETS["rna"])[k]
            a, b = _related(rng, alpha, n, m, 0.1) if k != 1 else (_rand(rng, alpha, n), _rand(rng, alpha, m))
            got, st = _score(engine, a, b, engine.Params(*prm_t))
            assert st["dna"] == 2 and st["variant"] & 4 and st["variant"] & 8192, st   # ring, three columns
            assert got == oracle_mod.score_linear(a, b, op), (prm_t, n, m)
    finally:
        engine.set_option("ring", -1)


def test_hepta_c5_size_acgtn(engine):
    """N = 2^20 with 1 % N (C5's shape, ring mode by size): the seven-letter ring kernel equals the
    byte path (hep = 0)."""
    rng = np.random.default_rng(1 << 20)
    a, b = engine.gen_pair(1 << 20, 1 << 20)
    a, b = a.copy(), b.copy()
    a[rng.random(1 << 20) < 0.01] = ord("N")
    b[rng.random(1 << 20) < 0.01] = ord("N")
    got = engine.SmithWatermanScoreCUDA(a, b)
    st = engine.last_stats()
    assert st["dna"] == 2 and st["variant"] & 4 and st["variant"] & HEP_BIT, st
    engine.set_option("hep", 0)
    ref = engine.SmithWatermanScoreCUDA(a, b)
    assert engine.last_stats()["dna"] == 0
    assert got == ref and got > 100000
