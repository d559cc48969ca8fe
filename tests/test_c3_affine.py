"""GPU parity of the batched Gotoh path (G_INIT != G_EXT) at config C3's size against the
reference-pinned goldens (main.cpp:54-66, lazySmith.cpp:27-41 at (2, -3, 5, 2)):

* C3_affine: all 1024 C3 pairs (seeds 8192 + k, N = 8192), uniform random DNA;
* C3_affine_similar: 1024 pairs oracle.similar_pair(8192 + k, 8192) with long alignments and
  indels of up to 32 bases, so E and F legs cross every strip edge of a duo.

Both are scored by the reference's own LazySmith built with these constants and by the oracle
(tests/golden/gen_pin.py --affine --npairs 1024 / --c3similar).  Each batch runs through the
automatic plan (the packed-u16 duo kernel, affine step, LDS hand-offs), through the device-arena
entry point the bench times, and on the int32 kernels (flow2 / flow3 step, a pair per
workgroup) that batches with scores >= 2^16 take.  Bit-exact integer equality."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

AFF = (2, -3, 5, 2)


@pytest.fixture(autouse=True)
def _defaults(engine):
    yield
    engine.set_option("mode", -1)
    engine.set_option("f2pwg", -1)
    engine.set_params(engine.Params())


def _c3_pairs(engine, c):
    N = c["N"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], N)
    return arena, [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]


def _similar_pairs(oracle_mod, c):
    return [oracle_mod.similar_pair(c["seed_base"] + k, c["N"]) for k in range(c["npairs"])]


def _auto_plan(engine, pairs, prm, want):
    got = engine.score_batch(pairs, prm)
    st = engine.last_stats()
    # the automatic plan: duo (mode 3), LDS hand-offs (variant 128), the general affine step (no bit 8)
    assert st["mode"] == 3 and st["variant"] & 128 and not st["variant"] & 8, st
    assert st["boundary_bytes"] == 0, st
    bad = [k for k in range(len(want)) if got[k] != want[k]]
    assert not bad, ("duo affine", bad[:8], [(got[k], want[k]) for k in bad[:8]])


def _int32_plan(engine, pairs, prm, want, pwg):
    """The int32 kernels: flow3's three-column affine ring step with a pair per workgroup (f3pwg 1,
    variant 32768) and flow2's one-column step (f3pwg 0)."""
    engine.set_option("mode", 5)
    engine.set_option("f2pwg", pwg)
    try:
        for f3pwg in (1, 0):
            engine.set_option("f3pwg", f3pwg)
            got = engine.score_batch(pairs, prm)
            st = engine.last_stats()
            assert st["mode"] == 5 and not st["variant"] & 8 and bool(st["variant"] & 32768) == bool(f3pwg), st
            bad = [k for k in range(len(want)) if got[k] != want[k]]
            assert not bad, ("int32 affine", pwg, f3pwg, bad[:8])
    finally:
        engine.set_option("f3pwg", 1)


def test_c3_affine_golden(engine, golden):
    """All 1024 C3 pairs at (2, -3, 5, 2) on the automatic plan and the int32 pair-per-workgroup
    kernel, against C3_affine (the reference's refvar LazySmith)."""
    c = golden("configs.json")["C3_affine"]
    assert c["npairs"] == 1024 and c["params"] == list(AFF)
    _, pairs = _c3_pairs(engine, c)
    prm = engine.Params(*AFF)
    _auto_plan(engine, pairs, prm, c["scores"])
    _int32_plan(engine, pairs, prm, c["scores"], 1)


def test_c3_affine_device_arena(engine, golden):
    """The bench's entry point: the C3 arena resident in HBM, sw_score_batch_device on a stream
    of its own, affine constants set with sw_set_params; two launches, same scores."""
    import torch
    c = golden("configs.json")["C3_affine"]
    N, P = c["N"], c["npairs"]
    arena, _ = _c3_pairs(engine, c)
    d_arena = torch.from_numpy(arena).cuda()
    scores = torch.zeros(P, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    engine.set_params(engine.Params(*AFF))
    for _ in range(2):
        scores.zero_()
        torch.cuda.synchronize()
        engine.score_batch_device(d_arena.data_ptr(), [2 * N * k for k in range(P)], [N] * P,
                                  [2 * N * k + N for k in range(P)], [N] * P, scores.data_ptr(), flags=1,
                                  stream=s.cuda_stream)
        s.synchronize()
        engine.stream_status(s.cuda_stream)
        assert scores.cpu().tolist() == c["scores"]
    st = engine.last_stats()
    assert st["mode"] == 3 and not st["variant"] & 8, st


def test_c3_affine_similar_golden(engine, golden, oracle_mod):
    """1024 E/F-heavy pairs of 8192 (scores ~10-12k, indels up to 32 bases) at (2, -3, 5, 2) on the
    automatic plan and the int32 kernel, against C3_affine_similar."""
    c = golden("configs.json")["C3_affine_similar"]
    assert c["npairs"] == 1024 and c["params"] == list(AFF)
    pairs = _similar_pairs(oracle_mod, c)
    prm = engine.Params(*AFF)
    for k in (0, 511, 1023):   # the generator itself, checked on a sample against the oracle
        assert oracle_mod.score_linear(*pairs[k], oracle_mod.Params(*AFF)) == c["scores"][k]
    _auto_plan(engine, pairs, prm, c["scores"])
    _int32_plan(engine, pairs, prm, c["scores"], 1)
