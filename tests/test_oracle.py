"""CPU: the oracle against the reference's own golden vectors and (in the build
container) against the reference's own main.cpp / lazySmith.cpp."""
import hashlib

import numpy as np
import pytest


def _sha(a, b):
    h = hashlib.sha256()
    h.update(np.asarray(a, np.uint8).tobytes()); h.update(b"|"); h.update(np.asarray(b, np.uint8).tobytes())
    return h.hexdigest()


def test_kats(oracle_mod, golden):
    g = golden("kat.json")
    for c in g["cases"]:
        a, b = c["seq1"], c["seq2"]
        assert oracle_mod.score_linear(a, b) == c["score"], (a[:20], b[:20])
        if len(a) * len(b) <= 4000 * 4000:
            assert oracle_mod.score_full(a, b) == c["score"]
    for c in g["byte_cases"]:
        a, b = bytes.fromhex(c["seq1_hex"]), bytes.fromhex(c["seq2_hex"])
        assert oracle_mod.score_full(a, b) == c["score"]


def test_published_seeded_sets(oracle_mod, golden):
    """cudaSmithM.cu:278-363 published scores, cudaCompareSmith.cu, CPUtesting.cpp."""
    for s in golden("seeded.json")["sets"]:
        st = oracle_mod.Stream(s["stream_seed"])
        for N, exp, h in zip(s["lengths"], s["scores"], s["sha256"]):
            if s["order"] == "interleaved":
                a, b = st.pair(N)
            else:
                a, b = st.seq(N), st.seq(N)
            assert _sha(a, b) == h
            if N <= 4096:
                assert oracle_mod.score_linear(a, b) == exp


def test_params_sets(oracle_mod, golden):
    for s in golden("params.json")["sets"]:
        p = oracle_mod.Params(*s["params"])
        for c in s["cases"][:8]:
            assert oracle_mod.score_full(c["seq1"], c["seq2"], p) == c["score"]
            assert oracle_mod.score_linear(c["seq1"], c["seq2"], p) == c["score"]


def test_config_c1(oracle_mod, golden):
    c = golden("configs.json")["C1"]
    a, b = oracle_mod.gen_pair(c["seed"], c["N"])
    assert _sha(a, b) == c["sha256"]
    assert oracle_mod.score_full(a, b) == c["score"] == 124


def test_wavefront_equals_linear(oracle_mod):
    rng = np.random.default_rng(5)
    for p in (oracle_mod.Params(), oracle_mod.Params(2, -3, 5, 2)):
        for _ in range(6):
            n, m = int(rng.integers(1, 700)), int(rng.integers(1, 700))
            a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)]
            b = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, m)]
            assert oracle_mod.score_wavefront(a, b, p, threads=4) == oracle_mod.score_linear(a, b, p)


def test_slabs_chain_to_linear(oracle_mod):
    """Column slabs chained through their (H, E) edges reproduce the whole pair:
    the max over slabs is score_linear, for any cut points (the multi-GPU slab
    checker itself, pinned to the lazySmith restatement)."""
    rng = np.random.default_rng(8)
    for p in (oracle_mod.Params(), oracle_mod.Params(2, -3, 5, 2), oracle_mod.Params(1, -1, 3, 1)):
        for _ in range(5):
            n, m = int(rng.integers(2, 900)), int(rng.integers(1, 600))
            a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)]
            b = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, m)]
            cuts = sorted(set([0, n] + [int(x) for x in rng.integers(1, n, 3)]))
            best, edge = 0, None
            for lo, hi in zip(cuts, cuts[1:]):
                s, edge = oracle_mod.slab(a[lo:hi], b, p, edge)
                assert s == oracle_mod.score_slab(a, b, lo, hi, p)[0]
                best = max(best, s)
            assert best == oracle_mod.score_linear(a, b, p), (p, n, m, cuts)


def test_restatement_vs_reference_build(oracle_mod):
    """Only where oracle/_ref exists (build container): the reference's own code."""
    if oracle_mod.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(11)
    for _ in range(60):
        n, m = int(rng.integers(1, 200)), int(rng.integers(1, 200))
        a = rng.integers(0, 256, n).astype(np.uint8)
        b = rng.integers(0, 256, m).astype(np.uint8)
        if rng.random() < 0.7:
            a = np.frombuffer(b"ACGT", np.uint8)[a % 4]; b = np.frombuffer(b"ACGT", np.uint8)[b % 4]
        r = oracle_mod.ref_score(a, b)
        assert oracle_mod.score_full(a, b) == r == oracle_mod.ref_score(a, b, which="lazy")
    for prm in (oracle_mod.Params(2, -3, 5, 2), oracle_mod.Params(1, -1, 3, 1)):
        if oracle_mod.ref_lib(prm) is None:
            continue
        for _ in range(30):
            n, m = int(rng.integers(1, 150)), int(rng.integers(1, 150))
            a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)]
            b = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, m)]
            assert oracle_mod.score_linear(a, b, prm) == oracle_mod.ref_score(a, b, prm)


def test_restatement_vs_reference_c3_size(oracle_mod, golden):
    """Eight C3-size pairs (N = 8192, seeds 8192..8199): the restatement, the
    reference's own LazySmith (lazySmith.cpp:15-69 compiled in place) and the
    committed C3/C4 golden agree (the goldens were generated by the restatement,
    swo_linear; this pins them to the reference at full config size)."""
    if oracle_mod.ref_lib() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    gold = golden("configs.json")["C3"]["scores"][:8]
    for k in range(8):
        a, b = oracle_mod.gen_pair(8192 + k, 8192)
        r = oracle_mod.ref_score(a, b, which="lazy")
        assert oracle_mod.score_linear(a, b) == r == gold[k], k


def test_restatement_vs_reference_long_affine(oracle_mod):
    """G_INIT != G_EXT on long pairs (3000-4000, similar sequences with indels, so
    long gaps run through E and F): restatement == param-substituted builds of the
    reference's main.cpp / lazySmith.cpp (oracle/Makefile refvar)."""
    rng = np.random.default_rng(44)
    for prm in oracle_mod.REFVAR_PARAMS:
        if oracle_mod.ref_lib(prm) is None:
            pytest.skip("refvar builds absent (make -C oracle refvar)")
        for n, m in ((3000, 3300), (4000, 3700)):
            a = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n)]
            b = np.resize(a, m).copy()
            mut = rng.random(m) < 0.08
            b[mut] = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, int(mut.sum()))]
            for cut in sorted(rng.integers(10, m - 40, 6)):   # indels of 1..30 bases
                ln = int(rng.integers(1, 30))
                b = np.concatenate([b[:cut], b[cut + ln:], b[:ln]])[:m] if rng.random() < 0.5 else \
                    np.concatenate([b[:cut], a[:ln], b[cut:]])[:m]
            exp = oracle_mod.ref_score(a, b, prm, which="lazy")
            assert oracle_mod.score_linear(a, b, prm) == exp == oracle_mod.ref_score(a, b, prm), (prm, n, m)


def test_config_c5_fixture(oracle_mod, golden):
    """The C5 golden (N = 2^20, seed 1048576) belongs to the generator's pair and was
    computed by two independent CPU engines that agree (tests/golden/gen_c5.py): the
    reference's own LazySmith compiled from lazySmith.cpp:15-69 (1 thread, 3.8 h) and
    the oracle's wavefront restatement; their result files are committed beside it."""
    c = golden("configs.json")["C5"]
    a, b = oracle_mod.gen_pair(c["seed"], c["N"])
    assert _sha(a, b) == c["sha256"]
    assert c["score"] == 119470
    assert any("reference LazySmith" in s for s in c["pinned_by"]), c["pinned_by"]
    assert any("swo_wavefront" in s for s in c["pinned_by"]), c["pinned_by"]
    for eng in ("ref", "wavefront"):
        r = golden("c5_%s.json" % eng)
        assert r["score"] == c["score"] and r["sha256"] == c["sha256"], (eng, r)


def test_config_c5_affine_fixture(oracle_mod, golden):
    """The C5 golden at the affine constants (2, -3, 5, 2): the same pair, scored by the
    reference's own LazySmith built with those constants (oracle/Makefile refvar, 1 thread,
    3.5 h) and by the oracle's wavefront restatement; both result files are committed."""
    c = golden("configs.json")["C5_affine"]
    a, b = oracle_mod.gen_pair(c["seed"], c["N"])
    assert _sha(a, b) == c["sha256"] and c["params"] == [2, -3, 5, 2]
    assert any("reference LazySmith" in s for s in c["pinned_by"]), c["pinned_by"]
    assert any("swo_wavefront" in s for s in c["pinned_by"]), c["pinned_by"]
    for eng in ("ref", "wavefront"):
        r = golden("c5_affine_%s.json" % eng)
        assert r["score"] == c["score"] and r["sha256"] == c["sha256"] and r["params"] == c["params"], (eng, r)


def test_config_c5_affine_similar_fixture(oracle_mod, golden):
    """The E/F-heavy C5-size golden: oracle.similar_pair(20, 2^20) at (2, -3, 5, 2), scored
    1392524 by the reference's own LazySmith built with those constants (1 thread, 2.8 h) and by
    the oracle's wavefront restatement (tests/golden/gen_pin.py --c5similar); both result files
    are committed and name the same pair."""
    c = golden("configs.json")["C5_affine_similar"]
    a, b = oracle_mod.similar_pair(20, c["N"])
    assert _sha(a, b) == c["sha256"] and c["params"] == [2, -3, 5, 2]
    assert any("reference LazySmith" in s for s in c["pinned_by"]), c["pinned_by"]
    assert any("swo_wavefront" in s for s in c["pinned_by"]), c["pinned_by"]
    for eng in ("ref", "wavefront"):
        r = golden("c5_affine_similar_%s.json" % eng)
        assert r["score"] == c["score"] and r["sha256"] == c["sha256"] and r["params"] == c["params"], (eng, r)
