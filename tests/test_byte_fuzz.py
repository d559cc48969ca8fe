"""Seeded fuzz of the engine's alphabet routing against the oracle: random byte alphabets of 1..12
values (so DNA, seven-letter and raw-byte paths all occur), random lengths, related and unrelated
sequences, random scoring constants over the engine's domain (MISMATCH = 0 and large MATCH - MISMATCH
among them, which keep byte batches off the duo kernels), as single pairs (host entry) and batches.
Bit-exact integer equality with the oracle (main.cpp SmithWatermanScore restated) on every case."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _alphabet(rng):
    k = int(rng.integers(1, 13))
    if rng.random() < 0.25:
        return np.frombuffer(b"ACGT", np.uint8)[: max(1, min(4, k))]
    return rng.choice(256, size=k, replace=False).astype(np.uint8)


def _seq_pair(rng, alpha, n, m):
    a = alpha[rng.integers(0, len(alpha), n)]
    if rng.random() < 0.5:
        b = alpha[rng.integers(0, len(alpha), m)]
    else:
        b = np.resize(a, m).copy()
        mut = rng.random(m) < rng.uniform(0.02, 0.3)
        b[mut] = alpha[rng.integers(0, len(alpha), int(mut.sum()))]
    return a, b


def _params(rng):
    mm = -int(rng.integers(0, 7))
    ma = int(rng.integers(max(1, mm), 6))
    gi = int(rng.integers(0, 9))
    ge = gi if rng.random() < 0.4 else int(rng.integers(0, 9))
    if rng.random() < 0.1:
        ma, mm = 90, -60          # MATCH - MISMATCH > 127: byte batches stay off the duo kernels
    return ma, mm, gi, ge


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_single_pairs(engine, oracle_mod, seed):
    rng = np.random.default_rng(1000 + seed)
    for _ in range(10):
        alpha = _alphabet(rng)
        a, b = _seq_pair(rng, alpha, int(rng.integers(1, 3000)), int(rng.integers(1, 3000)))
        prm = _params(rng)
        got = engine.score(a, b, engine.Params(*prm))
        exp = oracle_mod.score_linear(a, b, oracle_mod.Params(*prm))
        assert got == exp, (seed, len(alpha), len(a), len(b), prm, engine.last_stats())


@pytest.mark.parametrize("seed", range(4))
def test_fuzz_batches(engine, oracle_mod, seed):
    rng = np.random.default_rng(2000 + seed)
    for _ in range(3):
        alpha = _alphabet(rng)
        npairs = int(rng.integers(2, 90))
        pairs = [_seq_pair(rng, alpha, int(rng.integers(1, 2000)), int(rng.integers(1, 2000))) for _ in range(npairs)]
        prm = _params(rng)
        got = engine.score_batch(pairs, engine.Params(*prm))
        op = oracle_mod.Params(*prm)
        exp = [oracle_mod.score_linear(x, y, op) for x, y in pairs]
        assert got == exp, (seed, len(alpha), npairs, prm, engine.last_stats())
