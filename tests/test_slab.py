"""GPU: one pair split into column slabs -- the multi-GPU single-pair path
(SURVEY.md 8(f) f-1).  Slab r scores columns [bounds[r], bounds[r+1]) over all
rows; its left edge arrives as tagged granules written by slab r-1's kernel
straight into slab r's inflow buffer.  Here the slabs run as concurrent
launches on the one GPU of the box: from threads of one process (device
pointers) and from two processes through IPC-mapped inflow buffers (the
transport the ranks of a node use over xGMI).  The max over the slabs must
equal the oracle's score of the whole pair, bit-exact."""
import os
import socket
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ACGT = np.frombuffer(b"ACGT", np.uint8)


def _rand_dna(rng, n):
    return ACGT[rng.integers(0, 4, n)]


def _similar(rng, a, m, rate=0.06):
    b = np.resize(a, m).copy()
    mut = rng.random(m) < rate
    b[mut] = _rand_dna(rng, int(mut.sum()))
    return b


@pytest.fixture(autouse=True)
def _defaults(engine):
    engine.set_params(engine.Params())
    for k in ("W", "C", "bytes", "blocks", "orient"):
        engine.set_option(k, 0)
    engine.set_option("mode", -1)
    yield
    engine.set_params(engine.Params())
    for k in ("W", "C", "bytes", "blocks", "orient", "f2stream"):
        engine.set_option(k, 0)
    engine.set_option("mode", -1)


def _run_threads(engine, a, b, nslabs, flags, epoch=1):
    """Score (a, b) as nslabs concurrent slab launches, one host thread each."""
    import torch
    n, m = len(a), len(b)
    bounds = engine.slab_bounds(n, m, nslabs, flags)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    bufs = [engine.slab_alloc(m) for _ in range(nslabs)]   # bufs[r]: inflow of slab r (r > 0)
    scores = torch.full((nslabs,), -1, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    errs, stats = [None] * nslabs, [None] * nslabs
    ready = threading.Barrier(nslabs)
    # One stream for all slabs, slab r enqueued after slab r-1: kernels of one
    # process on one GPU are not guaranteed to run side by side (streams may share
    # a hardware queue), and a consumer running ahead of an unscheduled producer
    # would only time out.  Concurrent producer / consumer kernels are covered by
    # the two-process test below; ranks on different GPUs have no such coupling.
    shared = torch.cuda.Stream()
    launched = [[threading.Event() for _ in range(nslabs)] for _ in range(epoch + 1)]

    def work(r):
        try:
            # warm this thread's engine context with the same plan but no edges: its
            # buffers are then sized, and the edged launches below allocate nothing
            # (a hipFree while a neighbour slab's kernel waits on this one would
            # synchronise the device and stall both -- single process only)
            engine.score_slab_device(arena.data_ptr(), bounds[r], bounds[r + 1] - bounds[r], n, m, 0, 0, 0,
                                     scores.data_ptr() + 4 * r, flags)
            stream = shared
        except Exception as e:
            errs[r] = e
        ready.wait(timeout=60)
        try:
            for ep in range(1, epoch + 1):   # launches over the same buffers under fresh epochs
                if r > 0:
                    assert launched[ep][r - 1].wait(timeout=60), "producer slab never launched"
                if errs[r] is None:
                    engine.score_slab_device(arena.data_ptr(), bounds[r], bounds[r + 1] - bounds[r], n, m,
                                             bufs[r].ptr if r > 0 else 0, bufs[r + 1].ptr if r + 1 < nslabs else 0,
                                             ep, scores.data_ptr() + 4 * r, flags, stream.cuda_stream)
                launched[ep][r].set()
                if errs[r] is None:
                    engine.stream_status(stream.cuda_stream)   # synchronises, reports time-outs
                # every slab finished launch ep before any launch ep+1 rewrites an inflow
                # buffer (ColumnSlabs gets this from its all-reduce)
                ready.wait(timeout=60)
            stats[r] = engine.last_stats()
        except Exception as e:   # reported by the main thread
            errs[r] = e
            ready.abort()        # the other slabs stop waiting for this one
            for ev in launched:
                ev[r].set()

    import faulthandler
    faulthandler.dump_traceback_later(45)   # every thread's stack if a slab stalls
    try:
        th = [threading.Thread(target=work, args=(r,)) for r in range(nslabs)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th), "slab thread hung"
        real = [e for e in errs if e is not None and not isinstance(e, threading.BrokenBarrierError)]
        if real or any(e is not None for e in errs):
            raise (real or [e for e in errs if e is not None])[0]
        out = scores.cpu().tolist()
    finally:
        faulthandler.cancel_dump_traceback_later()
        torch.cuda.synchronize()
        for buf in bufs:
            buf.free()
    return out, bounds, stats


@pytest.mark.parametrize("nslabs", [2, 3])
def test_slabs_threads_every_kernel(engine, oracle_mod, nslabs):
    """Each grouped kernel as a slab: flow2 (DNA, rows in LDS), flow (DNA, constants
    outside flow2's byte range), chain (forced), and the raw-byte chain."""
    rng = np.random.default_rng(11 + nslabs)
    engine.set_option("blocks", 48)          # every slab's grid co-resides on the one GPU
    cases = [
        ("flow2", engine.Params(), engine.SW_FLAG_DNA, -1, 5),
        ("flow2-stream", engine.Params(2, -3, 5, 2), engine.SW_FLAG_DNA, -1, 5),   # codes streamed (C5 path)
        ("flow", engine.Params(2, -3, 130, 2), engine.SW_FLAG_DNA, -1, 4),
        ("chain", engine.Params(2, -3, 5, 2), engine.SW_FLAG_DNA, 2, 2),
        ("bytes", engine.Params(1, -1, 3, 1), engine.SW_FLAG_BYTES, -1, 2),
    ]
    for name, prm, flags, mode, want_mode in cases:
        engine.set_params(prm)
        engine.set_option("mode", mode)
        engine.set_option("f2stream", 1 if name == "flow2-stream" else 0)
        op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
        for n, m in ((nslabs * 600 + 77, 1500), (nslabs * 1300, 901)):
            a = _rand_dna(rng, n)
            b = _similar(rng, a, m) if m < n else _rand_dna(rng, m)
            if name == "bytes":
                a = a.copy()
                a[::97] = ord("N")
            exp = oracle_mod.score_linear(a, b, op)
            got, bounds, stats = _run_threads(engine, a, b, nslabs, flags)
            assert max(got) == exp, (name, n, m, got, exp, bounds)
            assert all(s["mode"] == want_mode for s in stats), (name, [s["mode"] for s in stats])
            # flow2 slabs run the slab kernel, which streams the row codes
            assert all(bool(s["variant"] & 2) == name.startswith("flow2") for s in stats), name
            # a slab reports max(0, max t) over its cells (t = diagonal + s): an H that
            # comes from a gap opened in an earlier slab is counted there, so a slab's
            # value is at most the oracle's max H over its columns, and the pair's
            # score is the max over the slabs
            for r in range(nslabs):
                lo, hi = bounds[r], bounds[r + 1]
                assert got[r] <= oracle_mod.score_slab(a, b, lo, hi, op)[0], (name, r, bounds)


@pytest.mark.parametrize("nslabs", [2, 3])
def test_slabs_ring_mode(engine, oracle_mod, nslabs):
    """The ring + slab instantiation (sw_flow2_kernel<C, STREAM, RING, SLAB, LIN>), the
    kernel the automatic plan runs for every C5 column slab: ring edges forced with
    512-row rings and 3 blocks per slab (several rounds of ~8 groups, the wrap ring
    every round, back-pressure since m > 512), with the linear-gap step, the affine
    step on the same constants (linear = 0) and G_INIT != G_EXT constants."""
    rng = np.random.default_rng(31 + nslabs)
    engine.set_option("ring", 1)
    engine.set_option("ring_rows", 512)
    engine.set_option("blocks", 3)
    try:
        for prm, lin in ((engine.Params(), -1), (engine.Params(), 0), (engine.Params(2, -3, 5, 2), -1)):
            engine.set_params(prm)
            engine.set_option("linear", lin)
            op = oracle_mod.Params(prm.match, prm.mismatch, prm.gap_init, prm.gap_ext)
            for n, m in ((nslabs * 2000 + 77, 1500), (nslabs * 1800, 2100)):
                a = _rand_dna(rng, n)
                b = _similar(rng, a, m) if m < n else _rand_dna(rng, m)
                exp = oracle_mod.score_linear(a, b, op)
                got, bounds, stats = _run_threads(engine, a, b, nslabs, engine.SW_FLAG_DNA)
                assert max(got) == exp, (prm, lin, n, m, got, exp, bounds)
                for s in stats:
                    assert s["mode"] == 5 and s["variant"] & 4 and s["variant"] & 2, s   # ring, streamed
                    assert bool(s["variant"] & 8) == (lin != 0 and prm.gap_init == prm.gap_ext), s
                    assert s["blocks"] == 3 and s["C"] == 64, s
    finally:
        engine.set_option("ring", -1)
        engine.set_option("ring_rows", 4096)
        engine.set_option("linear", -1)


def test_slab_long_alignment_crosses_every_edge(engine):
    """An identical pair: the optimal alignment runs the whole diagonal through
    every slab edge, so any lost or stale hand-off lowers the score; three
    launches reuse the inflow buffers under epochs 1, 2, 3."""
    rng = np.random.default_rng(5)
    a = _rand_dna(rng, 6000)
    engine.set_option("blocks", 64)
    got, _, _ = _run_threads(engine, a, a.copy(), 3, engine.SW_FLAG_DNA, epoch=3)
    assert got[-1] == 6000 and max(got) == 6000


def test_slab_errors(engine):
    import torch
    arena = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    sc = torch.zeros(1, dtype=torch.int32, device="cuda")
    buf = engine.slab_alloc(1000)
    try:
        with pytest.raises(engine.SwError):   # an outflow edge must end on a strip boundary
            engine.score_slab_device(arena.data_ptr(), 0, 100, 2048, 1000, 0, buf.ptr, 1, sc.data_ptr(),
                                     engine.SW_FLAG_BYTES)
        with pytest.raises(engine.SwError):   # epoch 0 is the never-written tag
            engine.score_slab_device(arena.data_ptr(), 0, 128, 2048, 1000, 0, buf.ptr, 0, sc.data_ptr(),
                                     engine.SW_FLAG_BYTES)
        with pytest.raises(engine.SwError):   # the alphabet must be stated
            engine.score_slab_device(arena.data_ptr(), 0, 128, 2048, 1000, 0, buf.ptr, 1, sc.data_ptr(), 0)
    finally:
        buf.free()
    assert engine.score(b"ACGT", b"ACGT") == 4   # engine still healthy


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ipc_worker(rank, world, port, n, m, seed, stream_codes, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import concurrentproject_amd as sw
        from concurrentproject_amd.dist import ColumnSlabs
        sw.set_option("timeout", 10)
        sw.set_option("blocks", 64)          # both ranks' grids fit the one GPU together
        sw.set_option("f2stream", stream_codes)
        a, b = sw.gen_pair(seed, n)
        b = b[:m]
        arena = torch.from_numpy(np.concatenate([a, b])).cuda()
        slabs = ColumnSlabs(n, m, sw.SW_FLAG_DNA)
        res = []
        for _ in range(2):   # the second launch reuses the buffers under a new epoch
            res.append(int(slabs.run(arena.data_ptr(), 0, n).item()))
        fine = slabs.inflow.fine_grained if slabs.inflow is not None else None
        bounds = slabs.bounds
        slabs.close()
        q.put((rank, res, bounds, fine, None))
    except Exception as e:
        q.put((rank, None, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("stream_codes", [0, 1])
def test_slabs_two_processes_ipc(oracle_mod, stream_codes):
    """Two ranks, one GPU: rank 0's kernel writes its right edge into rank 1's
    inflow buffer through an IPC mapping, as between the GPUs of a node; flow2
    with staged and with streamed row codes."""
    import torch.multiprocessing as mp
    n, m, seed = 8192, 3000, 8192
    a, b = oracle_mod.gen_pair(seed, n)
    exp = oracle_mod.score_linear(a, b[:m])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, 2, port, n, m, seed, stream_codes, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=240) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for rank, got, bounds, fine, err in res:
        assert err is None, (rank, err)
        assert got == [exp, exp], (rank, got, exp, bounds)
    # rank 1's inflow is exported for rank 0's kernel: fine-grained memory (sw_slab_alloc
    # refuses plain memory for an exported buffer), rank 0 has no inflow
    assert res[0][3] is None and res[1][3] is True, res
    print("slab IPC: bounds", res[0][2], "rank-1 inflow fine-grained:", res[1][3])
