"""GPU: flow2 ring mode (one long pair, group edges through per-block rings, O(m)
boundary state; sw_flow2.hip) against the oracle, and the
C5 pair (BASELINE configs[4], N = 2^20) against its committed golden."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", np.uint8)
OPTS = ("W", "C", "blocks", "orient", "f2stream", "f2_wgs", "f2w")


@pytest.fixture(autouse=True)
def _defaults(engine):
    def reset():
        engine.set_params(engine.Params())
        for k in OPTS:
            engine.set_option(k, 0)
        engine.set_option("mode", -1)
        engine.set_option("ring", -1)
        engine.set_option("ring_rows", 4096)
    reset()
    yield
    reset()


def _pairs(rng):
    out = []
    for n, m in [(253, 700), (1009, 513), (2017, 3001), (4096, 2600), (5000, 1200)]:
        a = ACGT[rng.integers(0, 4, n)]
        if rng.random() < 0.5:
            b = np.resize(a, m).copy()          # long diagonals through every group edge
            mut = rng.random(m) < 0.05
            b[mut] = ACGT[rng.integers(0, 4, int(mut.sum()))]
        else:
            b = ACGT[rng.integers(0, 4, m)]
        out.append((a, b))
    return out


def _strips(n, variant):
    """Strips of the single-pair kernel that ran: 189 columns (W3, variant 8192), 126 (W2, 16) or 63."""
    if variant & 8192:
        return 1 if n <= 192 else (n - 3 + 188) // 189
    if variant & 16:
        return (n - 2 + 125) // 126 if n > 128 else 1
    return (n - 1 + 62) // 63


@pytest.mark.parametrize("f2w", [2, 3])
def test_ring_mode_matches_oracle(engine, oracle_mod, f2w):
    """Forced ring mode on grids of 1, 2, 3 and 7 blocks (many rounds, the wrap
    ring used every round) and rings of 512 rows (rows wrap them several times),
    default and G_INIT != G_EXT constants.  Ring mode always runs the streamed-code
    kernel (finalize_mode sets f2_stream with ring; variant bit 2); the staged
    kernel and its loader wave are covered with linear edges
    (test_gpu_parity.py::test_flow2_loader_wave)."""
    rng = np.random.default_rng(91)
    pairs = _pairs(rng)
    engine.set_option("orient", 1)
    engine.set_option("mode", 5)
    engine.set_option("ring", 1)
    engine.set_option("f2w", f2w)   # two columns per lane (sw_flow2 / sw_flow3ra) or three (flow3 W3)
    for prm in (engine.Params(), engine.Params(2, -3, 5, 2), engine.Params(3, -2, 4, 4)):
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        exp = [oracle_mod.score_linear(a, b, op) for a, b in pairs]
        for blocks, rows in ((0, 4096), (1, 512), (2, 512), (3, 1024), (7, 512)):
            engine.set_option("blocks", blocks)
            engine.set_option("ring_rows", rows)
            got = []
            for a, b in pairs:
                got.append(engine.score(a, b, prm))
                st = engine.last_stats()
                groups = (_strips(len(a), st["variant"]) + 3) // 4
                assert st["mode"] == 5 and bool(st["variant"] & 4) == (groups > 1), st
                # f2w = 2 keeps the two-column ring kernels; f2w = 3 takes three columns in ring mode
                assert not (f2w == 2 and st["variant"] & 8192), st
                assert not (f2w == 3 and st["variant"] & 4) or st["variant"] & 8192, st
                # two columns per lane when the linear-gap step runs (G_INIT == G_EXT), and in ring
                # mode for the affine step too (flow3's sw_flow3ra_kernel, variant bit 1024)
                ring_aff = bool(st["variant"] & 4 and st["variant"] & 1024)
                assert bool(st["variant"] & 16) == (prm.gap_init == prm.gap_ext or ring_aff), st
                assert groups == 1 or st["variant"] & 2, st   # ring mode streams the row codes
            assert got == exp, (prm, blocks, rows)


def test_ring_matches_linear_edges(engine):
    """Ring and write-once edges give the same score on a pair of 240 groups."""
    a, b = engine.gen_pair(424242, 60000)
    engine.set_option("ring", 0)
    lin = engine.score(a, b)
    assert not engine.last_stats()["variant"] & 4
    engine.set_option("ring", 1)
    assert engine.score(a, b) == lin
    st = engine.last_stats()
    assert st["variant"] & 4 and st["boundary_bytes"] < 64 << 20, st


@pytest.mark.parametrize("f2w", [1, 2])
@pytest.mark.parametrize("wgs", [1, 2, 3, 4])
def test_ring_round_change(engine, wgs, f2w):
    """1588 groups at one column per lane (794 at two) over 256..1024 resident blocks
    (1..7 rounds): a block starts its next round while the consumer of its ring, one
    hop behind, still reads the last rows of the previous one.  The back-pressure
    check also covers a round's first R rows (before it did not, and N = 400000 at 2
    workgroups per CU timed out).  Ring edges at 1..4 workgroups per CU against
    write-once edges."""
    a, b = engine.gen_pair(400000, 400000)
    engine.set_option("f2w", f2w)
    engine.set_option("f2_wgs", wgs)
    engine.set_option("ring", 0)
    lin = engine.score(a, b)
    engine.set_option("ring", 1)
    got = engine.score(a, b)
    st = engine.last_stats()
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    items = st["items"]   # 4-strip groups: 1588 at one column per lane, 794 at two
    assert items == (1588 if f2w == 1 else 794) and bool(st["variant"] & 16) == (f2w == 2), st
    assert st["variant"] & 4 and st["blocks"] == min(items, wgs * cus), st
    assert got == lin > 0, (got, lin)


def test_config_c5_golden(engine, golden):
    """C5 (BASELINE configs[4]): N = 2^20, seed 1048576, scored from HBM through the
    device entry point with the automatic plan (flow2, streamed codes, ring edges:
    boundary state < 1 GB) and checked against the CPU golden (the reference's own
    LazySmith compiled from lazySmith.cpp:15-69, cross-checked by the oracle's
    wavefront restatement; tests/golden/gen_c5.py)."""
    import torch
    cfg = golden("configs.json")
    if "C5" not in cfg:
        pytest.fail("tests/golden/configs.json has no C5 golden")
    c = cfg["C5"]
    N = c["N"]
    a, b = engine.gen_pair(c["seed"], N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s.cuda_stream)
    engine.stream_status(s.cuda_stream)
    st = engine.last_stats()
    assert st["mode"] == 5 and st["variant"] & 4, st
    assert st["boundary_bytes"] < 1 << 30, st
    assert score.item() == c["score"]


def test_n_2pow21_ring(engine):
    """A pair of 2^21 (4.4e12 cells; write-once edges would need 279 GB): ring mode
    scores it, and the transposed problem (the other sequence across the lanes)
    gives the same score (size-independent property; no CPU golden at this size)."""
    import torch
    N = 1 << 21
    a, b = engine.gen_pair(2097152, N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    out = []
    for orient in (1, 2):
        engine.set_option("orient", orient)
        score = torch.full((1,), -1, dtype=torch.int32, device="cuda")
        s = torch.cuda.current_stream()
        engine.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1,
                                  stream=s.cuda_stream)
        engine.stream_status(s.cuda_stream)
        st = engine.last_stats()
        assert st["variant"] & 4 and st["boundary_bytes"] < 1 << 30, st
        out.append(score.item())
    assert out[0] == out[1] > 0, out
