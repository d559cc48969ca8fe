"""GPU parity: the flow2 kernel with a pair per workgroup (sw_flow2.hip PWG, option
f2pwg), the path of DNA batches whose scores need int32, against the oracle,
bit-exact.  Every hand-off of a pair goes through its workgroup's LDS rings, wave 3
to wave 0 of the next round included; the shapes cut the strips into rounds of 1-4
strips, rows around the 64-row chunk, both steps (two columns per lane with the
linear-gap step, one column with the affine step), grids smaller than the batch."""
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
            b = np.resize(a, m).copy()        # long diagonals through every strip and round edge
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
        engine.set_option("linear", -1)
        engine.set_option("f2w", 0)
        engine.set_option("f2pwg", -1)
        engine.set_option("f3pwg", 1)
    reset()
    yield
    reset()


# strips at two columns per lane: 1 (n <= 128), 2, 4, 5, 8, 9, 16 ...; rows below, at and
# around the 64-row chunk
SHAPES = [(1, 1), (5, 200), (128, 64), (129, 63), (254, 65), (255, 129), (504, 1000), (505, 127), (630, 700),
          (1009, 1), (1010, 2000), (1135, 333), (2017, 2100), (3000, 4097), (4096, 999), (8000, 8192)]


def test_pwg_forced_matches_oracle(engine, oracle_mod):
    """f2pwg = 1 with mode 5 on flow2's kernel (f3pwg = 0; flow3's three-column one: test_pwg3.py):
    ragged batch, linear-gap and affine constants, the automatic grid and grids of 1 and 3 workgroups
    (each runs many pairs)."""
    rng = np.random.default_rng(21)
    pairs = _pairs(rng, SHAPES)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("f2pwg", 1)
    engine.set_option("f3pwg", 0)
    for prm in (engine.Params(), engine.Params(2, -3, 5, 2), engine.Params(3, -2, 4, 4), engine.Params(1, 0, 0, 0)):
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        for blocks in (0, 1, 3):
            engine.set_option("blocks", blocks)
            assert engine.score_batch(pairs, prm) == exp, (prm, blocks)
            st = engine.last_stats()
            lin = prm.gap_init == prm.gap_ext
            assert st["mode"] == 5 and st["variant"] & 32 and st["C"] == 64, st
            assert bool(st["variant"] & 16) == lin and bool(st["variant"] & 8) == lin, st
            assert st["items"] == len(pairs) and st["boundary_bytes"] == 0, st
        # one column per lane at the linear-gap constants (f2w = 1): the affine PWG step
        if prm.gap_init == prm.gap_ext:
            engine.set_option("f2w", 1)
            engine.set_option("blocks", 2)
            assert engine.score_batch(pairs, prm) == exp, (prm, "f2w=1")
            st = engine.last_stats()
            assert st["variant"] & 32 and not st["variant"] & 24, st
            engine.set_option("f2w", 0)


def test_pwg_is_the_int32_batch_path(engine, oracle_mod):
    """A DNA batch whose scores may reach 2^16 (MATCH * min(n, m) + MATCH > 65535), as
    many pairs as CUs or more, takes PWG automatically; fewer pairs than CUs take the
    flow2 item claim; f2pwg = 0 falls back to the pair-per-workgroup strip kernel."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(22)
    shapes = [(int(rng.integers(680, 720)), int(rng.integers(680, 720))) for _ in range(cus + 40)]
    pairs = _pairs(rng, shapes)
    prm = engine.Params(100, -20, 20, 20)        # 100 * 680 + 100 > 65535: no 16-bit duos
    op = oracle_mod.Params(100, -20, 20, 20)
    exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
    assert max(exp) > 30000
    assert engine.score_batch(pairs, prm) == exp
    st = engine.last_stats()
    assert st["mode"] == 5 and st["variant"] & 32, st
    assert engine.score_batch(pairs[:6], prm) == exp[:6]
    st = engine.last_stats()
    assert st["mode"] == 5 and not st["variant"] & 32 and st["variant"] & 2, st   # item claim, streamed
    engine.set_option("f2pwg", 0)
    assert engine.score_batch(pairs[:40], prm) == exp[:40]
    assert engine.last_stats()["mode"] != 5


def test_batch_kernel_by_batch_size(engine, oracle_mod):
    """Automatic choice for DNA batches that fit 16 bits: fewer pairs than CUs -> the
    flow2 item claim, fewer than 2 per CU -> a pair per workgroup, more -> duos; the
    same scores every way."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    rng = np.random.default_rng(23)
    shapes = [(int(rng.integers(560, 640)), int(rng.integers(560, 640))) for _ in range(2 * cus + 16)]
    pairs = _pairs(rng, shapes)
    exp = [oracle_mod.score_linear(a, b) for a, b in pairs]
    for count, mode, pwg in ((cus // 2, 5, False), (cus + 16, 5, True), (2 * cus + 16, 3, False)):
        assert engine.score_batch(pairs[:count]) == exp[:count], count
        st = engine.last_stats()
        assert st["mode"] == mode and bool(st["variant"] & 32) == pwg, (count, st)
    engine.set_option("mode", 3)   # the duo kernel forced on the smallest batch
    assert engine.score_batch(pairs[:cus // 2]) == exp[:cus // 2]
    assert engine.last_stats()["mode"] == 3


def test_pwg_config_c3_on_int32(engine, golden):
    """The C3 batch (1024 pairs N = 8192, seeds 8192+k) on the int32 PWG kernel against
    its golden.  Its scores fit 16 bits, so the duo kernel would take it; the int32 path
    is forced (mode 5, f2pwg 1)."""
    import torch
    c = golden("configs.json")["C3"]
    N, P, exp = c["N"], c["npairs"], c["scores"]
    host = engine.gen_batch(c["seed_base"], P, N)
    arena = torch.from_numpy(host).cuda()
    scores = torch.full((P,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.set_option("mode", 5)
    engine.set_option("f2pwg", 1)
    engine.set_option("f3pwg", 0)   # flow2's kernel (flow3's: test_pwg3.py)
    engine.score_batch_device(arena.data_ptr(), [2 * N * k for k in range(P)], [N] * P,
                              [2 * N * k + N for k in range(P)], [N] * P, scores.data_ptr(), flags=1,
                              stream=s.cuda_stream)
    engine.stream_status(s.cuda_stream)
    st = engine.last_stats()
    assert st["mode"] == 5 and st["variant"] & 32 and st["variant"] & 16, st
    assert scores.cpu().tolist() == exp[:P]
