"""GPU parity: the general affine (Gotoh) step on flow3 (sw_flow3.hip sw_flow3a_kernel: one
column per lane, hand-scheduled chunk loops from tools/gen_flow3.py gen_role_aff), bit-exact
against the oracle (main.cpp:54-66 / lazySmith.cpp:27-41 restated) and against flow2's affine
step (option f3a = 0) on the same inputs.  Ragged shapes around the 63-column strip stride, the
252-column groups and the 32-row chunks cover every strip role (no inflow / LDS inflow x no
outflow / LDS / 16-B granules); grids of 1-3 workgroups run the groups in rounds through the
loader.  Constant sets with G_INIT > G_EXT, G_INIT < G_EXT, G_INIT == G_EXT forced affine
(linear = 0) and zero gaps; C2 in full against the reference-pinned goldens."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)
AFF = (2, -3, 5, 2)


def _pairs(rng, shapes):
    out = []
    for n, m in shapes:
        a = ACGT[rng.integers(0, 4, n)]
        b = ACGT[rng.integers(0, 4, m)]
        if rng.random() < 0.6 and m > 10:
            b = np.resize(a, m).copy()        # long diagonals and gaps through every strip edge
            mut = rng.random(m) < 0.06
            b[mut] = ACGT[rng.integers(0, 4, int(mut.sum()))]
            for cut in sorted(rng.integers(0, m, 3)):
                ln = int(rng.integers(1, 40))
                b = np.concatenate([b[:cut], b[cut + ln:], b[:ln]])[:m] if rng.random() < 0.5 else \
                    np.concatenate([b[:cut], ACGT[rng.integers(0, 4, ln)], b[cut:]])[:m]
        out.append((np.ascontiguousarray(a), np.ascontiguousarray(b)))
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
        engine.set_option("f3a", 1)
        engine.set_option("f3hl", 1)
    reset()
    yield
    reset()


# rows around the 32-row chunks and the ring's 512 rows, columns around the 63-column strips
# and 252-column groups (1, 2, 4, 5, 8, 9 strips)
SHAPES = [(1, 1), (1, 200), (200, 1), (2, 5), (63, 64), (64, 63), (65, 33), (126, 95), (127, 96), (128, 97),
          (252, 255), (253, 256), (254, 257), (505, 511), (506, 512), (1000, 513), (1009, 1000), (1135, 1100),
          (2017, 2100), (4096, 3000), (5041, 777)]
PARAMS = ((2, -3, 5, 2), (1, -1, 3, 1), (1, -1, 1, 3), (3, -2, 4, 1), (1, 0, 0, 0))


def test_flow3a_ragged(engine, oracle_mod):
    rng = np.random.default_rng(51)
    pairs = _pairs(rng, SHAPES)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)      # flow2 planning for every shape (single strips included)
    engine.set_option("W", 1)
    for C, hl in ((32, 1), (32, 0), (16, 0)):
        engine.set_option("C", C)
        engine.set_option("f3hl", hl)
        for prm in PARAMS:
            p = engine.Params(*prm)
            op = oracle_mod.Params(*prm)
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            if prm[2] == prm[3]:
                engine.set_option("linear", 0)   # the affine step at G_INIT == G_EXT
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, p))
                st = engine.last_stats()
                assert st["mode"] == 5 and st["variant"] & 1024 and not st["variant"] & (8 | 16 | 64), st
                assert bool(st["variant"] & 512) == bool(hl) and st["C"] == C, st
            assert got == exp, (prm, C, hl)
            assert engine.score_batch(pairs, p) == exp, (prm, C, hl)
            for blocks in (1, 2, 3):
                engine.set_option("blocks", blocks)
                assert engine.score_batch(pairs, p) == exp, (prm, blocks, C, hl)
            engine.set_option("blocks", 0)
            engine.set_option("linear", -1)
    engine.set_option("C", 0)


def test_flow3a_matches_flow2(engine):
    """The same launches on flow2's affine step (option f3a = 0) give the same scores."""
    rng = np.random.default_rng(52)
    pairs = _pairs(rng, [(3001, 2999), (6000, 1500), (1500, 6000), (777, 9000)])
    p = engine.Params(*AFF)
    engine.set_option("mode", 5)
    engine.set_option("W", 1)
    got3 = engine.score_batch(pairs, p)
    assert engine.last_stats()["variant"] & 1024
    engine.set_option("f3a", 0)
    got2 = engine.score_batch(pairs, p)
    assert not engine.last_stats()["variant"] & 1024
    assert got3 == got2


def _device_score(engine, a, b):
    import torch
    N, M = len(a), len(b)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [M], score.data_ptr(), flags=1, stream=s.cuda_stream)
    engine.stream_status(s.cuda_stream)
    return score.item()


def test_flow3a_config_c2_affine(engine, golden):
    """C2 (N = 65536, seed 65536) with G_INIT != G_EXT on the default plan (flow3a, 32-row chunks,
    half-chunk links) and at 16-row chunks, against the golden of the reference's own LazySmith
    built with those constants."""
    g = golden("configs.json")["C2_affine"]
    a, b = engine.gen_pair(g["seed"], g["N"])
    engine.set_params(engine.Params(*g["params"]))
    for C in (0, 16):
        engine.set_option("C", C)
        engine.set_option("f3hl", 1 if C == 0 else 0)
        assert _device_score(engine, a, b) == g["score"]
        st = engine.last_stats()
        assert st["variant"] & 1024 and st["C"] == (C or 32), st


def test_flow3a_c2_similar(engine, oracle_mod, golden):
    """A C2-size pair with long alignments and long gaps (oracle.similar_pair) at (2, -3, 5, 2):
    the score runs through long E and F legs across every strip and group edge."""
    g = golden("configs.json")["C2_affine_similar"]
    a, b = oracle_mod.similar_pair(7, g["N"])
    engine.set_params(engine.Params(*g["params"]))
    assert _device_score(engine, a, b) == g["score"]
    assert engine.last_stats()["variant"] & 1024
    engine.set_option("f3a", 0)
    assert _device_score(engine, a, b) == g["score"]     # flow2's affine step too


def test_flow3a_linear0_c2(engine, golden):
    """The default constants with the linear-gap identity off (linear = 0): the affine step on the
    C2 pair gives the C2 golden."""
    g = golden("configs.json")["C2"]
    a, b = engine.gen_pair(g["seed"], g["N"])
    engine.set_option("linear", 0)
    assert _device_score(engine, a, b) == g["score"]
    assert engine.last_stats()["variant"] & 1024


# ---- ring mode (sw_flow3.hip sw_flow3ra_kernel: two columns per lane, C = 64, streamed row
# codes, group edges through per-block rings of 16-B granules; the C5 organisation)

@pytest.fixture
def _ring_reset(engine):
    yield
    engine.set_option("ring", -1)
    engine.set_option("ring_rows", 4096)
    engine.set_option("blocks", 0)
    engine.set_option("f2w", 0)


@pytest.mark.parametrize("f2w", [2, 3])
def test_flow3ra_ring_parity(engine, oracle_mod, _ring_reset, f2w):
    """Ring mode forced on grids of 1, 2, 3 and 7 blocks with 512-row rings (many rounds, the
    wrap ring every round), rows around the 64-row chunk pairs, the affine constant sets; two
    columns per lane (f2w = 2: sw_flow3ra_kernel) and three (f2w = 3: sw_flow3ra3_kernel)."""
    rng = np.random.default_rng(53)
    pairs = _pairs(rng, [(253, 700), (1009, 513), (2017, 3001), (4096, 2600), (5000, 1200), (9000, 2000),
                         (3025, 127), (2521, 129), (600, 64), (130, 3000)])
    engine.set_option("orient", 1)
    for prm in PARAMS:
        p = engine.Params(*prm)
        op = oracle_mod.Params(*prm)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        engine.set_option("linear", 0 if prm[2] == prm[3] else -1)
        for blocks, rows in ((0, 4096), (1, 512), (2, 512), (3, 1024), (7, 512)):
            engine.set_option("ring", 1)
            engine.set_option("f2w", f2w)
            engine.set_option("blocks", blocks)
            engine.set_option("ring_rows", rows)
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, p))
                st = engine.last_stats()
                if f2w == 3 and st["variant"] & 8192:
                    strips = 1 if len(a) <= 192 else (len(a) - 3 + 188) // 189
                else:
                    strips = (len(a) - 2 + 125) // 126 if len(a) > 128 else 1
                groups = (strips + 3) // 4
                if groups > 1:
                    assert st["variant"] & 1024 and st["variant"] & 4 and st["variant"] & 16 and st["C"] == 64, st
                    assert not st["variant"] & (8 | 64), st
                    # the kernel the option names: sw_flow3ra_kernel (f2w = 2) or sw_flow3ra3_kernel (3)
                    assert bool(st["variant"] & 8192) == (f2w == 3), st
            assert got == exp, (prm, blocks, rows)
    engine.set_option("linear", -1)


def test_flow3ra_matches_flow2(engine, _ring_reset):
    """A 2^17 pair in ring mode (affine constants): flow3's two-column affine kernel and flow2's
    one-column affine step (f3a = 0) give the same score."""
    import torch
    N = 1 << 17
    a, b = engine.gen_pair(N, N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.set_params(engine.Params(*AFF))
    engine.set_option("ring", 1)
    out = []
    for f3a in (1, 0):
        engine.set_option("f3a", f3a)
        engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1,
                                  stream=s.cuda_stream)
        engine.stream_status(s.cuda_stream)
        st = engine.last_stats()
        assert bool(st["variant"] & 1024) == bool(f3a) and st["variant"] & 4, st
        out.append(score.item())
    assert out[0] == out[1] > 0


@pytest.mark.parametrize("f2w", [2, 3])
def test_flow3ra_ring_c2_similar(engine, oracle_mod, golden, _ring_reset, f2w):
    """The E/F-heavy C2-size pair (C2_affine_similar, 91137: long gaps through every strip, group
    and ring hand-off) in ring mode on the two- and three-column affine ring kernels, on grids of
    1-3 workgroups with 512-row rings (the wrap ring every round)."""
    g = golden("configs.json")["C2_affine_similar"]
    a, b = oracle_mod.similar_pair(7, g["N"])
    engine.set_params(engine.Params(*g["params"]))
    engine.set_option("ring", 1)
    engine.set_option("f2w", f2w)
    engine.set_option("ring_rows", 512)
    for blocks in (1, 2, 3):
        engine.set_option("blocks", blocks)
        assert _device_score(engine, a, b) == g["score"], (f2w, blocks)
        st = engine.last_stats()
        assert st["variant"] & 1024 and st["variant"] & 4 and bool(st["variant"] & 8192) == (f2w == 3), st


def test_flow3ra_c2_similar_slabs(engine, oracle_mod, golden):
    """The same pair cut into 2 and 4 column slabs (the affine slab kernels, peer edges through
    slab buffers, threads on one GPU): the max over the slabs is the golden."""
    from test_slab import _run_threads
    g = golden("configs.json")["C2_affine_similar"]
    a, b = oracle_mod.similar_pair(7, g["N"])
    engine.set_params(engine.Params(*g["params"]))
    engine.set_option("blocks", 32)          # every slab's grid co-resides on the one GPU
    try:
        for nslabs in (2, 4):
            got, bounds, stats = _run_threads(engine, a, b, nslabs, engine.SW_FLAG_DNA)
            assert max(got) == g["score"], (nslabs, got, bounds)
            for st in stats:
                assert st["variant"] & 1024 and st["variant"] & 2048, st
    finally:
        engine.set_option("blocks", 0)


def test_flow3ra_config_c5_affine_similar(engine, golden, oracle_mod):
    """An E/F-heavy pair at C5 size (oracle.similar_pair(20, 2^20), alignments of ~1.5M with
    indels of up to 4096 bases) at (2, -3, 5, 2) on the default plan (flow3 W3 ring affine),
    against C5_affine_similar (the oracle's pthread wavefront and the reference's LazySmith)."""
    g = golden("configs.json")["C5_affine_similar"]
    assert any(p.startswith("reference LazySmith") for p in g["pinned_by"]), g["pinned_by"]
    a, b = oracle_mod.similar_pair(20, g["N"])
    engine.set_params(engine.Params(*g["params"]))
    assert _device_score(engine, a, b) == g["score"]
    st = engine.last_stats()
    assert st["variant"] & 1024 and st["variant"] & 4 and st["variant"] & 8192, st
    assert st["boundary_bytes"] < 1 << 30, st


def test_flow3ra_config_c5_affine(engine, golden):
    """C5 (N = 2^20, seed 1048576) with G_INIT != G_EXT on the default plan (flow3 ring affine),
    against its golden; the ring keeps the boundary state O(N) (< 1 GB)."""
    cfg = golden("configs.json")
    if "C5_affine" not in cfg:
        pytest.skip("C5_affine golden not generated yet (tests/golden/gen_pin.py --c5affine)")
    g = cfg["C5_affine"]
    a, b = engine.gen_pair(g["seed"], g["N"])
    engine.set_params(engine.Params(*g["params"]))
    assert _device_score(engine, a, b) == g["score"]
    st = engine.last_stats()
    assert st["variant"] & 1024 and st["variant"] & 4 and st["boundary_bytes"] < 1 << 30, st


# ---- the pool loops (option f3pool = 1, tools/gen_flow3.py gen_pool: no I/O rotation, inflow rows
# broadcast from LDS into a 32-step register pool, outflow stored by lane 63; off by default:
# measured slower) -- kept bit-exact on both steps

def test_flow3_pool_option(engine, oracle_mod, golden):
    rng = np.random.default_rng(57)
    pairs = _pairs(rng, SHAPES)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("C", 32)
    engine.set_option("f3pool", 1)
    try:
        for prm in (AFF, (1, -1, 1, 1), (1, -1, 3, 1)):
            lin = prm[2] == prm[3]
            engine.set_option("W", 0 if lin else 1)   # linear-gap: flow3's two-column kernel
            engine.set_option("f2w", 2 if lin else 0)
            p = engine.Params(*prm)
            op = oracle_mod.Params(*prm)
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, p))
                st = engine.last_stats()
                assert st["variant"] & 4096 and st["variant"] & 512 and st["C"] == 32, (prm, st)
                assert bool(st["variant"] & 64) == lin and bool(st["variant"] & 1024) != lin, (prm, st)
            assert got == exp, prm
            for blocks in (1, 3):
                engine.set_option("blocks", blocks)
                assert engine.score_batch(pairs, p) == exp, (prm, blocks)
            engine.set_option("blocks", 0)
        for k in ("W", "f2w", "C", "orient"):
            engine.set_option(k, 0)
        engine.set_option("mode", -1)
        for key in ("C2", "C2_affine"):
            g = golden("configs.json")[key]
            a, b = engine.gen_pair(g["seed"], g["N"])
            engine.set_params(engine.Params(*g.get("params", (1, -1, 1, 1))))
            assert _device_score(engine, a, b) == g["score"], key
            assert engine.last_stats()["variant"] & 4096, key
    finally:
        engine.set_option("f3pool", 0)
