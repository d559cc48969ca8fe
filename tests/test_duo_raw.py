"""GPU parity of byte batches on the duo kernels (sw_kernels.hip SENT_RAW: the penalty from the
raw bytes, one XOR and one v_pk_min_u16 per position, option duo_raw) against the oracle and
against the byte-path strip kernels (duo_raw = 0) on the same inputs.  Bit-exact integer
equality.  main.cpp:28-33 scores by byte equality, so any byte value is a symbol.

Covered: protein (20 letters), all 256 byte values (0x00, 0x7F, 0xFF among them: the sentinel
encodings live in the low byte of each half, the data in the high one), ACGT with N, mixed
case, a two-letter alphabet of the sentinel bytes themselves; ragged duos (dead columns and
sentinel rows inside a duo), W = 1 / 2 / 4 / 8, the LDS-table, DPP-code and granule kernels, the
f16-max3 and u16 forms, linear-gap and affine steps; the host's fallbacks (MISMATCH >= 0,
MATCH - MISMATCH > 127) keep the strip kernels; a C3-shaped protein batch in full against the
byte path; a protein database search (f-4)."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PROTEIN = np.frombuffer(b"ACDEFGHIKLMNPQRSTVWY", np.uint8)
ALPHABETS = {
    "protein": PROTEIN,
    "bytes": np.arange(256, dtype=np.uint8),
    "acgtn": np.frombuffer(b"ACGTN", np.uint8),
    "mixed": np.frombuffer(b"ACGTacgt", np.uint8),
    "sentinels": np.array([0x00, 0x7F, 0xFF, 0x80], np.uint8),
}
PARAMS = [(1, -1, 1, 1), (2, -3, 5, 2), (3, -1, 4, 1), (5, -4, 8, 3)]


def _rand(rng, alpha, n):
    return alpha[rng.integers(0, len(alpha), n)]


def _related(rng, alpha, n, m, p=0.1):
    """b: a's first m symbols (wrapped) with a fraction p replaced and a few indels, so
    alignments run long and the E / F legs cross strip edges."""
    a = _rand(rng, alpha, n)
    b = np.resize(a, m).copy()
    mut = rng.random(m) < p
    b[mut] = _rand(rng, alpha, int(mut.sum()))
    for _ in range(3):
        if m > 40:
            k = int(rng.integers(10, m - 10))
            b = np.concatenate([b[:k], _rand(rng, alpha, int(rng.integers(1, 6))), b[k:]])[:m]
    return a, b


@pytest.fixture(autouse=True)
def _defaults(engine):
    yield
    for k in ("blocks", "W", "C"):
        engine.set_option(k, 0)
    engine.set_option("mode", -1)
    engine.set_option("duo_lds", 1)
    engine.set_option("duo_tab", 1)
    engine.set_option("duo16", 1)
    engine.set_option("duo_raw", 1)
    engine.set_option("linear", -1)


def _oracle(oracle_mod, pairs, prm_t):
    op = oracle_mod.Params(*prm_t)
    return [oracle_mod.score_linear(a, b, op) for a, b in pairs]


def _duo(engine, pairs, prm, W=8):
    engine.set_option("mode", 3)
    engine.set_option("W", W)
    engine.set_option("C", 64 if W >= 4 else 32)
    got = engine.score_batch(pairs, prm)
    st = engine.last_stats()
    assert st["mode"] == 3 and st["dna"] == 0 and st["W"] == W, st
    return got, st


def _pairs(rng, alpha, k=16):
    ns = [100, 512, 513, 1100, 1600, 2100, 2700]
    ms = [1, 63, 64, 65, 511, 575, 1000, 2049]
    out = []
    for i in range(k):
        n, m = ns[i % len(ns)], ms[(3 * i) % len(ms)]
        out.append(_related(rng, alpha, n, m) if i % 3 else (_rand(rng, alpha, n), _rand(rng, alpha, m)))
    return out


@pytest.mark.parametrize("alpha", sorted(ALPHABETS))
@pytest.mark.parametrize("prm_t", PARAMS)
def test_duo_raw_alphabets(engine, oracle_mod, alpha, prm_t):
    """Ragged duos of every alphabet on the LDS kernels (table and DPP codes, W = 8 / 4), the
    linear-gap and affine steps: equal to the oracle."""
    rng = np.random.default_rng(zlib.crc32(repr((alpha, prm_t)).encode()))
    pairs = _pairs(rng, ALPHABETS[alpha])
    prm = engine.Params(*prm_t)
    exp = _oracle(oracle_mod, pairs, prm_t)
    assert max(exp) > 0
    for lin in ((-1, 0) if prm_t[2] == prm_t[3] else (-1,)):
        engine.set_option("linear", lin)
        for W in (8, 4):
            for tab in (1, 0):
                engine.set_option("duo_tab", tab)
                got, st = _duo(engine, pairs, prm, W)
                assert st["variant"] & 128, st
                assert got == exp, (alpha, prm_t, lin, W, tab)


@pytest.mark.parametrize("prm_t", [(1, -1, 1, 1), (2, -3, 5, 2)])
def test_duo_raw_kernel_forms(engine, oracle_mod, prm_t):
    """The granule duo kernel (duo_lds = 0), the u16-max form (duo16 = 0), W = 1 / 2 at C = 32 and
    grids of 1-3 workgroups over many duos: the same scores as the oracle."""
    rng = np.random.default_rng(77 + prm_t[0])
    pairs = [_related(rng, PROTEIN, int(rng.integers(50, 3000)), int(rng.integers(1, 2500))) for _ in range(22)]
    pairs += [(_rand(rng, ALPHABETS["bytes"], 700), _rand(rng, ALPHABETS["bytes"], 900))]
    prm = engine.Params(*prm_t)
    exp = _oracle(oracle_mod, pairs, prm_t)
    engine.set_option("duo_lds", 0)
    got, st = _duo(engine, pairs, prm, 8)
    assert not st["variant"] & 128 and got == exp
    engine.set_option("duo_lds", 1)
    engine.set_option("duo16", 0)
    got, st = _duo(engine, pairs, prm, 8)
    assert not st["variant"] & 1 and got == exp
    engine.set_option("duo16", 1)
    for W in (1, 2):
        got, st = _duo(engine, pairs, prm, W)
        assert got == exp, W
    for blocks in (1, 2, 3):
        engine.set_option("blocks", blocks)
        got, _ = _duo(engine, pairs, prm, 8)
        assert got == exp, blocks


def test_duo_raw_automatic_plan_and_fallbacks(engine, oracle_mod):
    """Without forcing: a protein batch of 300 pairs runs on the duo kernel; parameters outside the
    RAW encoding (MISMATCH >= 0, MATCH - MISMATCH > 127) and duo_raw = 0 keep the strip kernels;
    all equal the oracle."""
    rng = np.random.default_rng(5)
    pairs = [_related(rng, PROTEIN, int(rng.integers(400, 1500)), int(rng.integers(400, 1500))) for _ in range(300)]
    for prm_t, duo in (((1, -1, 1, 1), True), ((2, -3, 5, 2), True), ((2, 0, 3, 1), False), ((100, -30, 40, 10), False)):
        exp = _oracle(oracle_mod, pairs[:40], prm_t)
        got = engine.score_batch(pairs, engine.Params(*prm_t))
        st = engine.last_stats()
        assert (st["mode"] == 3) == duo and st["dna"] == 0, (prm_t, st)
        assert got[:40] == exp, prm_t
    engine.set_option("duo_raw", 0)
    got0 = engine.score_batch(pairs)
    assert engine.last_stats()["mode"] != 3
    engine.set_option("duo_raw", 1)
    assert engine.score_batch(pairs) == got0


def test_duo_raw_c3_shaped_protein(engine, oracle_mod):
    """1024 protein pairs of 8192 (C3's shape) on the automatic plan (the duo LDS-table kernel):
    equal to the byte-path strip kernels (duo_raw = 0) on every pair and to the oracle on a sample."""
    rng = np.random.default_rng(8192)
    pairs = []
    for k in range(1024):
        pairs.append(_related(rng, PROTEIN, 8192, 8192, 0.3) if k % 4 == 0 else
                     (_rand(rng, PROTEIN, 8192), _rand(rng, PROTEIN, 8192)))
    got = engine.score_batch(pairs)
    st = engine.last_stats()
    assert st["mode"] == 3 and st["dna"] == 0 and st["variant"] & 256, st
    engine.set_option("duo_raw", 0)
    ref = engine.score_batch(pairs)
    assert engine.last_stats()["mode"] != 3
    assert got == ref
    op = oracle_mod.Params(1, -1, 1, 1)
    for k in (0, 1, 4, 511, 1020, 1023):
        assert got[k] == oracle_mod.score_linear(pairs[k][0], pairs[k][1], op), k
    assert max(got) > 1000   # the related pairs align end to end


def test_duo_raw_database_search(engine, oracle_mod):
    """f-4: a protein query against a FASTA of ragged protein records (SwissProt-style), through
    sw_db_search: the duo kernel scores every record, equal to the oracle."""
    from concurrentproject_amd.db import Database
    rng = np.random.default_rng(11)
    recs = [_rand(rng, PROTEIN, int(rng.integers(100, 2500))) for _ in range(700)]
    q = _rand(rng, PROTEIN, 1000)
    recs[17] = np.concatenate([recs[17][:100], q[20:700], recs[17][100:]])
    fasta = b"".join(b">p%d desc\n" % i + r.tobytes() + b"\n" for i, r in enumerate(recs))
    db = Database.from_fasta(fasta)
    try:
        sc = db.search(q)
        st = engine.last_stats()
        assert st["mode"] == 3 and st["dna"] == 0, st
        op = oracle_mod.Params(1, -1, 1, 1)
        exp = [oracle_mod.score_linear(q, r, op) for r in recs]
        assert list(sc) == exp
        assert int(np.argmax(sc)) == 17
    finally:
        db.close()
