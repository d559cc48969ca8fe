"""GPU parity: the HIP engine (through the C-ABI) against the oracle and the
committed golden fixtures.  Bit-exact integer equality everywhere."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)


def _rand_dna(rng, n):
    return ACGT[rng.integers(0, 4, n)]


@pytest.fixture(autouse=True)
def _defaults(engine):
    engine.set_params(engine.Params())
    for k in ("W", "C", "bytes", "blocks", "orient"):
        engine.set_option(k, 0)
    engine.set_option("mode", -1)
    yield
    engine.set_params(engine.Params())
    for k in ("W", "C", "bytes", "blocks", "orient", "f2w"):
        engine.set_option(k, 0)
    engine.set_option("mode", -1)


def test_kats_every_entry_point(engine, golden):
    g = golden("kat.json")
    fns = (engine.SequentialSmithWatermanScoreGPU, engine.SmithWatermanLazyGPU,
           engine.SmithWatermanScoreCUDA, engine.SmithDiagonalGPU)
    for c in g["cases"]:
        for f in fns:
            assert f(c["seq1"], c["seq2"]) == c["score"], (f.__name__, c["seq1"][:16], c["seq2"][:16])
    got = engine.score_batch([(c["seq1"], c["seq2"]) for c in g["cases"]])
    assert got == [c["score"] for c in g["cases"]]


def test_raw_byte_cases(engine, golden):
    g = golden("kat.json")["byte_cases"]
    pairs = [(bytes.fromhex(c["seq1_hex"]), bytes.fromhex(c["seq2_hex"])) for c in g]
    for (a, b), c in zip(pairs, g):
        assert engine.score(a, b) == c["score"]
    assert engine.score_batch(pairs) == [c["score"] for c in g]


def _regen(oracle_mod, s):
    st = oracle_mod.Stream(s["stream_seed"])
    out = []
    for N in s["lengths"]:
        if s["order"] == "interleaved":
            out.append(st.pair(N))
        else:
            out.append((st.seq(N), st.seq(N)))
    return out


def test_published_seeded_sets(engine, oracle_mod, golden):
    """cudaSmithM.cu:278-363 (published), cudaCompareSmith.cu:122-141, CPUtesting.cpp:131-142."""
    for s in golden("seeded.json")["sets"]:
        pairs = _regen(oracle_mod, s)
        assert [engine.SmithWatermanScoreCUDA(a, b) for a, b in pairs] == s["scores"], s["name"]
        assert engine.score_batch(pairs) == s["scores"], s["name"]


def test_testlazygpu_set(engine, oracle_mod, golden):
    """testLazyGPU_CPU.cu:231-243: 20 pairs, N = 5000..24000."""
    s = golden("seeded_lazygpu.json")["sets"][0]
    pairs = _regen(oracle_mod, s)
    assert [engine.SmithWatermanLazyGPU(a, b) for a, b in pairs] == s["scores"]
    assert engine.score_batch(pairs) == s["scores"]


def test_params_sets(engine, golden):
    """G_INIT != G_EXT and other constants (checked in the build container against
    param-substituted builds of the reference's main.cpp / lazySmith.cpp)."""
    for s in golden("params.json")["sets"]:
        p = engine.Params(*s["params"])
        pairs = [(c["seq1"], c["seq2"]) for c in s["cases"]]
        exp = [c["score"] for c in s["cases"]]
        assert [engine.score(a, b, p) for a, b in pairs] == exp, p
        assert engine.score_batch(pairs, p) == exp, p


def test_config_c1(engine, golden):
    c = golden("configs.json")["C1"]
    a, b = engine.gen_pair(c["seed"], c["N"])
    assert engine.SmithWatermanScoreCUDA(a, b) == c["score"] == 124


def test_config_c2_single_pair_65536(engine, golden):
    c = golden("configs.json")["C2"]
    a, b = engine.gen_pair(c["seed"], c["N"])
    assert engine.SmithWatermanScoreCUDA(a, b) == c["score"] == 7458
    # symmetric: the transposed problem gives the same score
    assert engine.SmithWatermanScoreCUDA(b, a) == c["score"]
    # every grid organisation and a wider strip agree at full size
    for mode in (0, 1, 2, 4, 5):
        engine.set_option("mode", mode)
        assert engine.SmithWatermanScoreCUDA(a, b) == c["score"], mode
    engine.set_option("mode", -1)
    assert engine.last_stats()["mode"] == 5   # the automatic plan for C2 is the flow2 kernel
    engine.set_option("mode", 5)
    for C in (16, 64):
        engine.set_option("C", C)
        assert engine.SmithWatermanScoreCUDA(a, b) == c["score"], C
    engine.set_option("C", 0)
    # the affine step on the default constants (the automatic plan takes the exact
    # linear-gap step, G_INIT == G_EXT) agrees at full size
    engine.set_option("linear", 0)
    assert engine.SmithWatermanScoreCUDA(a, b) == c["score"]
    assert not engine.last_stats()["variant"] & 8
    engine.set_option("linear", -1)
    assert engine.SmithWatermanScoreCUDA(a, b) == c["score"]
    assert engine.last_stats()["variant"] & 8
    engine.set_option("mode", -1)
    engine.set_option("W", 4)
    assert engine.SmithWatermanScoreCUDA(a, b) == c["score"]


def test_config_c3_batch_1024(engine, golden):
    c = golden("configs.json")["C3"]
    arena = engine.gen_batch(c["seed_base"], c["npairs"], c["N"])
    N = c["N"]
    pairs = [(arena[2 * N * k:2 * N * k + N], arena[2 * N * k + N:2 * N * (k + 1)]) for k in range(c["npairs"])]
    assert engine.score_batch(pairs) == c["scores"]
    assert engine.last_stats()["variant"] & 8          # the linear-gap duo step (G_INIT == G_EXT)
    engine.set_option("linear", 0)                     # and the affine duo step
    try:
        assert engine.score_batch(pairs) == c["scores"]
        assert not engine.last_stats()["variant"] & 8
    finally:
        engine.set_option("linear", -1)


def test_config_c4_batch_8192_device(engine, golden):
    """C4: 8192 pairs of N=8192 (seeds 8192+k) scored from one HBM arena through
    the device entry point; every score against the committed CPU golden."""
    import torch
    c = golden("configs.json")["C4"]
    N, P = c["N"], c["npairs"]
    arena = torch.from_numpy(engine.gen_batch(c["seed_base"], P, N)).cuda()
    scores = torch.full((P,), -1, dtype=torch.int32, device="cuda")
    offs_a = [2 * N * k for k in range(P)]
    offs_b = [2 * N * k + N for k in range(P)]
    s = torch.cuda.current_stream()
    engine.score_batch_device(arena.data_ptr(), offs_a, [N] * P, offs_b, [N] * P, scores.data_ptr(),
                              flags=1, stream=s.cuda_stream)
    torch.cuda.synchronize()
    engine.stream_status(s.cuda_stream)
    assert scores.cpu().tolist() == c["scores"]


def test_every_variant_ragged(engine, oracle_mod):
    """Each (W, C) kernel variant, DNA and raw-byte paths, on ragged shapes around
    the strip widths 64*W and chunk sizes, in one batch and one at a time."""
    rng = np.random.default_rng(2024)
    shapes = [(1, 1), (1, 300), (300, 1), (63, 64), (64, 63), (65, 129), (127, 128), (128, 127),
              (129, 255), (255, 257), (511, 513), (1024, 1000), (2049, 300), (300, 2049), (700, 3000)]
    pairs = []
    for n, m in shapes:
        a = _rand_dna(rng, n)
        b = _rand_dna(rng, m)
        if rng.random() < 0.5 and m > 10:   # similar pairs: long alignments cross strips
            b = np.resize(a, m).copy()
            mut = rng.random(m) < 0.08
            b[mut] = _rand_dna(rng, int(mut.sum()))
        pairs.append((a, b))
    for prm in (engine.Params(), engine.Params(2, -3, 5, 2), engine.Params(1, -1, 3, 1)):
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        for W, C in ((1, 16), (1, 32), (2, 32), (4, 64), (8, 64)):
            engine.set_option("W", W)
            engine.set_option("C", C)
            for force_bytes in (0, 1):
                engine.set_option("bytes", force_bytes)
                # independent strips, workgroup per pair, lock-step chain, packed u16 duos (DNA only)
                for mode in ((0, 1, 2) if force_bytes else (0, 1, 2, 3, 4)):
                    engine.set_option("mode", mode)
                    assert engine.score_batch(pairs, prm) == exp, (W, C, force_bytes, mode, prm)
                    for (a, b), e in list(zip(pairs, exp))[::4]:
                        assert engine.score(a, b, prm) == e, (W, C, force_bytes, mode, len(a), len(b))
                engine.set_option("mode", -1)


def test_flow2_ragged(engine, oracle_mod):
    """The single-pair flow2 kernel (overlapping 64-column strips, W=1, DNA) on
    ragged shapes around its 63-column stride, the 4-strip workgroups and the
    chunk sizes; several pairs per launch; a one-workgroup grid; params whose
    s + G_INIT leaves the signed byte fall back (auto) or fail (forced)."""
    rng = np.random.default_rng(77)
    shapes = [(1, 1), (1, 200), (200, 1), (63, 63), (64, 64), (65, 65), (126, 127), (127, 126), (128, 300),
              (252, 253), (253, 252), (255, 1000), (256, 17), (505, 505), (1000, 64), (2017, 2100), (4096, 4000)]
    pairs = []
    for n, m in shapes:
        a = _rand_dna(rng, n)
        b = _rand_dna(rng, m)
        if rng.random() < 0.5 and m > 10:
            b = np.resize(a, m).copy()
            mut = rng.random(m) < 0.05
            b[mut] = _rand_dna(rng, int(mut.sum()))
        pairs.append((a, b))
    engine.set_option("orient", 1)   # keep (n, m) as given: seq1 across the lanes
    try:
        for prm in (engine.Params(), engine.Params(2, -3, 5, 2), engine.Params(1, -1, 3, 1), engine.Params(1, 0, 0, 0),
                    engine.Params(60, -120, 67, 9), engine.Params(2, -3, 4, 4)):
            op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            engine.set_option("mode", 5)
            for C in (16, 32, 64):
                engine.set_option("C", C)
                # G_INIT == G_EXT: the linear-gap step (auto) at two columns per lane (auto) and, at
                # C = 32 / 64, at one (f2w = 1); the affine step (linear = 0).  C = 16 has the linear
                # step only at two columns per lane (the flow3 kernel)
                lin_ok = prm.gap_init == prm.gap_ext
                for lin, f2w in (((-1, 0), (-1, 1), (0, 0)) if lin_ok else ((-1, 0),)):
                    engine.set_option("linear", lin)
                    engine.set_option("f2w", f2w)
                    got = [engine.score(a, b, prm) for a, b in pairs]
                    assert got == exp, (C, prm, lin, f2w)
                    st = engine.last_stats()
                    assert st["mode"] == 5
                    lin_step = lin == -1 and lin_ok and (C != 16 or f2w == 0)
                    assert bool(st["variant"] & 8) == lin_step, st
                    assert bool(st["variant"] & 16) == (lin_step and f2w == 0), st
                    assert engine.score_batch(pairs, prm) == exp, (C, prm, lin, f2w)
                engine.set_option("linear", -1)
                engine.set_option("f2w", 0)
            engine.set_option("C", 0)
            engine.set_option("blocks", 1)
            assert engine.score_batch(pairs, prm) == exp, prm
            engine.set_option("blocks", 0)
            engine.set_option("mode", -1)
        # s + G_INIT > 127: the automatic plan uses another kernel, a forced flow2 reports an error
        prm = engine.Params(100, -1, 40, 1)
        a, b = pairs[-1]
        e = oracle_mod.score_linear(a, b, oracle_mod.Params(100, -1, 40, 1))
        assert engine.score(a, b, prm) == e
        assert engine.last_stats()["mode"] != 5
        engine.set_option("mode", 5)
        with pytest.raises(RuntimeError):
            engine.score(a, b, prm)
    finally:
        engine.set_option("mode", -1)
        engine.set_option("C", 0)
        engine.set_option("blocks", 0)
        engine.set_option("orient", 0)


def test_flow2_loader_wave(engine, oracle_mod):
    """The staged flow2 kernel's loader wave (a fifth wave that moves a workgroup's
    inflow granules into LDS for wave 0): pairs of many 4-strip groups on grids of
    1, 2, 3 and 7 workgroups (a group's producer ran on another or the same
    workgroup, or finished long before), row counts around the loader's 64-row
    window, several pairs per launch, linear-gap and affine steps."""
    rng = np.random.default_rng(2024)
    shapes = [(1100, 63), (1100, 64), (1100, 65), (2000, 127), (2000, 129), (3000, 1000), (4096, 2049)]
    pairs = [(_rand_dna(rng, n), _rand_dna(rng, m)) for n, m in shapes]
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    try:
        for prm in (engine.Params(), engine.Params(2, -3, 5, 2)):
            op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            for f2w in ((0, 1) if prm.gap_init == prm.gap_ext else (0,)):   # two / one column(s) per lane
                engine.set_option("f2w", f2w)
                for blocks in (1, 2, 3, 7, 0):
                    engine.set_option("blocks", blocks)
                    assert engine.score_batch(pairs, prm) == exp, (prm, blocks, f2w)
                    st = engine.last_stats()
                    assert st["mode"] == 5 and not st["variant"] & 2, st   # the staged kernel
            engine.set_option("f2w", 0)
            assert [engine.score(a, b, prm) for a, b in pairs] == exp, prm
    finally:
        engine.set_option("mode", -1)
        engine.set_option("blocks", 0)
        engine.set_option("orient", 0)


def test_flow2_loader_wave_timeout(engine, oracle_mod):
    """A producer group that never publishes (test option stall_item: flow2's compute waves skip
    item 0) makes the next group's loader wave and wave 0 wait in vain: their bounded spins expire,
    the launch reports ERR_TIMEOUT (SwError) within seconds instead of hanging, and the engine
    scores the next launch correctly.  Staged flow2 kernel, one column per lane, affine step."""
    import time
    rng = np.random.default_rng(77)
    a, b = _rand_dna(rng, 2000), _rand_dna(rng, 500)       # 32 strips: 8 groups, loader in groups 1..7
    prm = engine.Params(2, -3, 5, 2)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("f3a", 0)                             # flow2's affine step (staged, loader wave)
    engine.set_option("timeout", 1)
    try:
        engine.set_option("stall_item", 0)
        assert engine.get_option("stall_item") == 0
        t0 = time.time()
        with pytest.raises(engine.SwError):
            engine.score(a, b, prm)
        assert time.time() - t0 < 60
        st = engine.last_stats()
        assert st["mode"] == 5 and not st["variant"] & (2 | 64 | 1024), st   # flow2 staged, no flow3
        engine.set_option("stall_item", -1)
        op = oracle_mod.Params(2, -3, 5, 2)
        assert engine.score(a, b, prm) == oracle_mod.score_linear(a, b, op)
    finally:
        engine.set_option("stall_item", -1)
        engine.set_option("timeout", 5)
        engine.set_option("f3a", 1)
        engine.set_option("mode", -1)
        engine.set_option("orient", 0)


def test_flow2_streamed_rows(engine, oracle_mod):
    """flow2 with the row codes streamed through per-wave LDS rings (rows too long
    to stage, the C5 path): forced on the ragged flow2 shapes and chosen
    automatically for a pair whose 200000 rows exceed the LDS."""
    rng = np.random.default_rng(78)
    shapes = [(1, 1), (1, 300), (300, 1), (63, 63), (64, 64), (65, 65), (127, 126), (128, 300), (253, 252),
              (255, 1000), (256, 17), (1000, 64), (2017, 2100), (4096, 4000)]
    pairs = []
    for n, m in shapes:
        a = _rand_dna(rng, n)
        b = _rand_dna(rng, m)
        if rng.random() < 0.5 and m > 10:
            b = np.resize(a, m).copy()
            mut = rng.random(m) < 0.05
            b[mut] = _rand_dna(rng, int(mut.sum()))
        pairs.append((a, b))
    engine.set_option("orient", 1)
    engine.set_option("f2stream", 1)
    try:
        for prm in (engine.Params(), engine.Params(2, -3, 5, 2), engine.Params(60, -120, 67, 9)):
            op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            engine.set_option("mode", 5)
            for C in (16, 32, 64):
                engine.set_option("C", C)
                for f2w in ((0, 1) if prm.gap_init == prm.gap_ext and C > 16 else (0,)):
                    engine.set_option("f2w", f2w)
                    assert [engine.score(a, b, prm) for a, b in pairs] == exp, (C, prm, f2w)
                    assert engine.last_stats()["variant"] & 2
                    assert engine.score_batch(pairs, prm) == exp, (C, prm, f2w)
                engine.set_option("f2w", 0)
            engine.set_option("C", 0)
            engine.set_option("mode", -1)
        engine.set_option("f2stream", 0)
        # long rows: automatic flow2 (W = 1 for 700 columns) with streamed codes
        a = _rand_dna(rng, 700)
        b = _similar_rows(rng, a, 200000)
        e = oracle_mod.score_linear(a, b)
        assert engine.score(a, b) == e
        st = engine.last_stats()
        assert st["mode"] == 5 and st["variant"] & 2, st
    finally:
        engine.set_option("f2stream", 0)
        engine.set_option("mode", -1)
        engine.set_option("C", 0)
        engine.set_option("orient", 0)


def _similar_rows(rng, a, m):
    """m rows that repeat `a` with 5% point mutations (long local alignments)."""
    b = np.resize(a, m).copy()
    mut = rng.random(m) < 0.05
    b[mut] = _rand_dna(rng, int(mut.sum()))
    return b


def test_edges(engine, oracle_mod):
    assert engine.SmithWatermanScoreCUDA(b"", b"ACGT") == 0
    assert engine.SmithWatermanScoreCUDA(b"ACGT", b"") == 0
    assert engine.score_batch([(b"", b""), (b"A", b"A"), (b"", b"A")]) == [0, 1, 0]
    a = b"A" * 5000
    assert engine.SmithWatermanScoreCUDA(a, a) == 5000
    assert engine.SmithWatermanScoreCUDA(b"A" * 3135, b"T" * 3135) == 0
    # non-ACGT bytes: case-sensitive raw byte equality (main.cpp:28-33)
    assert engine.score(b"acgt", b"ACGT") == 0
    assert engine.score(bytes([0, 255, 0, 255]), bytes([0, 255, 0, 255])) == 4
    # identical long sequences: score = length (long diagonal through every strip)
    rng = np.random.default_rng(3)
    s = _rand_dna(rng, 20000)
    assert engine.score(s, s) == 20000
    # rectangular single pairs, both orientations
    x, y = _rand_dna(rng, 9000), _rand_dna(rng, 700)
    e = oracle_mod.score_linear(x, y)
    assert engine.score(x, y) == engine.score(y, x) == e


def test_linear_entry_point_semantics(engine, oracle_mod):
    """SmithDiagonalGPU is linear-gap (G_EXT := G_INIT), SmithDiagonalGPU.cu:59-66."""
    rng = np.random.default_rng(9)
    engine.set_params(engine.Params(2, -3, 5, 2))
    for _ in range(5):
        a, b = _rand_dna(rng, int(rng.integers(50, 900))), _rand_dna(rng, int(rng.integers(50, 900)))
        assert engine.SmithDiagonalGPU(a, b) == oracle_mod.score_linear(a, b, oracle_mod.Params(2, -3, 5, 5))
        assert engine.SmithWatermanScoreCUDA(a, b) == oracle_mod.score_linear(a, b, oracle_mod.Params(2, -3, 5, 2))


def test_device_resident_batch(engine, oracle_mod):
    import torch
    rng = np.random.default_rng(17)
    seqs, offs, pairs = [], [], []
    off = 0
    for _ in range(40):
        a, b = _rand_dna(rng, int(rng.integers(1, 1500))), _rand_dna(rng, int(rng.integers(1, 1500)))
        pairs.append((a, b))
        for s in (a, b):
            offs.append(off); seqs.append(s); off += len(s)
    arena = torch.from_numpy(np.concatenate(seqs)).cuda()
    scores = torch.full((40,), -7, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    alen = [len(a) for a, _ in pairs]; blen = [len(b) for _, b in pairs]
    for flags in (0, 1, 2):
        engine.score_batch_device(arena.data_ptr(), offs[0::2], alen, offs[1::2], blen, scores.data_ptr(),
                                  flags=flags, stream=stream)
        engine.stream_status(stream)
        exp = [oracle_mod.score_linear(a, b) for a, b in pairs]
        assert scores.cpu().tolist() == exp, flags


def test_errors_are_reported(engine):
    with pytest.raises(engine.SwError):
        engine.score(b"ACGT", b"ACGT", engine.Params(1, 2, 1, 1))     # positive mismatch
    with pytest.raises(engine.SwError):
        engine.score(b"ACGT", b"ACGT", engine.Params(1, -1, -2, 1))   # negative gap
    assert engine.score(b"ACGT", b"ACGT") == 4                       # engine still healthy


def test_duo_batches(engine, oracle_mod):
    """Packed 16-bit duo kernel: odd batch sizes, ragged shapes padded inside a
    duo, several constants; chosen automatically for DNA batches."""
    rng = np.random.default_rng(77)
    for prm, lin in ((engine.Params(), -1), (engine.Params(), 0), (engine.Params(2, -3, 5, 2), -1),
                     (engine.Params(3, -1, 4, 1), -1), (engine.Params(3, -2, 5, 5), -1)):
        # G_INIT == G_EXT: the exact linear-gap duo step unless linear = 0
        engine.set_option("linear", lin)
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        for npairs in (1, 2, 3, 7):
            pairs = []
            for _ in range(npairs):
                n, m = int(rng.integers(200, 2600)), int(rng.integers(200, 2600))
                a = _rand_dna(rng, n)
                b = np.resize(a, m).copy() if rng.random() < 0.5 else _rand_dna(rng, m)
                mut = rng.random(m) < 0.1
                b[mut] = _rand_dna(rng, int(mut.sum()))
                pairs.append((a, b))
            exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
            engine.set_option("mode", 3)
            assert engine.score_batch(pairs, prm) == exp, (prm, npairs, lin)
            st = engine.last_stats()
            assert bool(st["variant"] & 8) == (lin == -1 and prm.gap_init == prm.gap_ext and st["variant"] & 1), st
            engine.set_option("mode", -1)
            assert engine.score_batch(pairs, prm) == exp, (prm, npairs, lin)
    engine.set_option("linear", -1)


def test_duo_f16_max3_boundary(engine, oracle_mod):
    """The duo's v_pk_maximum3_f16 variant (u16 halves read as f16 bit patterns) is
    used while MATCH*(min(n,m)+1) <= 0x7BFF; identical pairs put the running max,
    H and t right at that edge, one base more takes the u16-max duo.  Both agree
    with the oracle, and the variant agrees with duo16=0 on random batches."""
    rng = np.random.default_rng(21)
    s = _rand_dna(rng, 31743)
    engine.set_option("mode", 3)
    try:
        assert engine.score_batch([(s[:31742], s[:31742]), (s[:9000], s[:9000])]) == [31742, 9000]
        assert engine.score_batch([(s, s), (s[:10], s[:10])]) == [31743, 10]
        pairs = []
        for _ in range(9):
            n, m = int(rng.integers(300, 3000)), int(rng.integers(300, 3000))
            a = _rand_dna(rng, n)
            b = np.resize(a, m).copy()
            mut = rng.random(m) < 0.15
            b[mut] = _rand_dna(rng, int(mut.sum()))
            pairs.append((a, b))
        for prm in (engine.Params(), engine.Params(3, -2, 7, 1)):
            exp = [oracle_mod.score_linear(a, b, oracle_mod.Params(*prm.__dict__.values())) for a, b in pairs]
            for flag in (1, 0):
                engine.set_option("duo16", flag)
                assert engine.score_batch(pairs, prm) == exp, (prm, flag)
    finally:
        engine.set_option("duo16", 1)
        engine.set_option("mode", -1)


def test_duo_16bit_boundary(engine):
    """H + MATCH must fit 16 bits: 65534 identical bases is the largest exact duo case;
    one more forces the int32 kernels (auto) or an error (forced duo)."""
    rng = np.random.default_rng(5)
    s = _rand_dna(rng, 65535)
    engine.set_option("mode", 3)
    pairs = [(s[:65534], s[:65534]), (s[:40000], s[:40000])]
    assert engine.score_batch(pairs) == [65534, 40000]
    with pytest.raises(engine.SwError):
        engine.score_batch([(s, s), (s[:10], s[:10])])
    engine.set_option("mode", -1)
    assert engine.score_batch([(s, s), (s[:10], s[:10])]) == [65535, 10]
