#!/usr/bin/env python3
"""Benchmark of the MI355X Smith-Waterman score path (BASELINE.json metric: GCUPS).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload auto|pair|batch|slab]

Ranks: one process per GPU.  Under torchrun (RANK/WORLD_SIZE set) this process
is one rank; standalone with --gpus N > 1 it checks that N GPUs are visible
(exit 2 otherwise), starts N ranks of itself (concurrentproject_amd.launch:
rank r on device r, MASTER_ADDR 127.0.0.1) and exits with their status.  The
ranks form an "nccl" (RCCL) group; `n_gpus` is its world size.

Workloads (BASELINE.json configs; synthetic uniform {A,C,G,T}, generator of
cudaSmithM.cu:200-212, sequences resident in HBM before the timed region):
  pair   C2: one pair N=65536 (seed 65536), one launch per step.  With N ranks
         the global batch is N such pairs (seeds 65536+rank), one per rank, the
         per-pair scores gathered to rank 0 over RCCL every step (weak scaling
         of the same per-GPU work as the N=1 line).
  batch  C3/C4: 1024 pairs of N=8192 per GPU; rank r scores pairs
         [1024r, 1024r+1024) (seeds 8192+k), then the per-pair int32 scores are
         gathered to rank 0 with RCCL every step.  8 ranks = config C4.
  slab   C5: one pair N=2^20 (seed 1048576); with N ranks its columns are cut
         into one slab per rank (dist.ColumnSlabs); per-rank kernel times and
         the pipeline fill are reported beside `value`.
  auto   `value` is the pair workload at every N (C2 at N=1: configs[1], the
         metric's single-GPU config), so the 1/2/4/8 series compares the same
         per-GPU work.  The batched config is measured after it on the same
         ranks and reported as "batch_c3" (N=1) or "batch_c4" (N>1: 1024 pairs
         per GPU, C4 at N=8; north_star's >= 7.5x is stated on batched pairs).
A step is one full pass of the hot path over the step's input; `value` is the
whole-job GCUPS (sum of n*m over all ranks' pairs / max-over-ranks time).

Roofline: the kernels keep H/E/F in registers, so the bound
that applies is VALU issue, not HBM.  `roofline.achieved` = VALU lane-ops of one
launch (rocprofv3 SQ_INSTS_VALU x 64, profiles/pmc_<workload>.json, valid only
for the same libswmi355.so, checked by sha256) / the launch time measured here;
`peak` = 256 CU x 4 SIMD x 64 lanes / 2 cycles x 2.4 GHz.  For the single pair
`critical_path_frac` = (m + 63 x strips) x the step time measured in this run
(strip 0 of a traced launch) / the launch time: the wavefront's own bound, since
strip s+1 cannot start a row sooner than 63 steps after strip s (n + m at one
column per lane, m + n/2 at two).  `traffic` = HBM bytes per launch from
the FETCH_SIZE / WRITE_SIZE passes of the same profile.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
ALGO_BYTES_PER_CELL = 12       # int32 H, E, F produced per cell
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 2
# cycles (32 lanes/clk, MI355X_MICROARCH.md "v_fma_f32 2 cyc (SIMD-32)"), 2.4 GHz
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12   # T lane-ops/s = 78.64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); standalone N > 1 spawns them, under torchrun it must equal WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="auto", choices=["auto", "pair", "batch", "slab"])
    ap.add_argument("--slab-of", type=int, default=0,
                    help="slab workload, one GPU: time slab 0 of a K-way column split alone (per-rank cost)")
    ap.add_argument("--n", type=int, default=0, help="override sequence length")
    ap.add_argument("--pairs-per-gpu", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="N=1 auto: skip the extra C3 / affine / C5 measurements")
    ap.add_argument("--no-c5", action="store_true", help="N=1 auto: skip the extra C5 (N=2^20) launches")
    ap.add_argument("--W", type=int, default=0)
    ap.add_argument("--C", type=int, default=0)
    ap.add_argument("--mode", type=int, default=-1, help="engine option 'mode' (-1 = automatic plan)")
    ap.add_argument("--params", default="1,-1,1,1", help="MATCH,MISMATCH,G_INIT,G_EXT")
    ap.add_argument("--opt", action="append", default=[], help="engine option key=value (sw_set_option)")
    return ap.parse_args()


def load_golden():
    try:
        with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
            return json.load(f)
    except OSError:
        return {}


def lib_sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def host_cores():
    """(threads the CPU leg may use, what the host reports).  The GPU box gives one
    GPU's job a share of its cores: OMP_NUM_THREADS (16 there) caps the pool."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return (min(avail, cap) if cap > 0 else avail), {"nproc": os.cpu_count(), "affinity": avail,
                                                      "omp_num_threads": cap or None}


def cpu_baseline(kind: str, n: int, budget_s: float, params):
    """The reference's sequential CPU path (main.cpp:40-90, full matrix) restated in
    oracle/sw_oracle.c, timed on a bounded sample of the same workload."""
    import oracle  # the checker / baseline leg only
    p = oracle.Params(*params)
    threads, host = host_cores()
    if kind == "pair":
        a, b = oracle.gen_pair(65536, 65536) if n == 65536 else oracle.gen_pair(65536, n)
        rows, spent, cells, t_tot = 128, 0.0, 0, 0.0
        while True:
            t0 = time.perf_counter()
            oracle.score_full(a, b[:rows], p)      # main.cpp layout on the first `rows` rows
            dt = time.perf_counter() - t0
            cells += rows * len(a); t_tot += dt; spent += dt
            if spent > budget_s or rows >= len(b):
                break
            rows = min(len(b), rows * 2)
        return {"value": cells / t_tot / 1e9, "unit": "GCUPS", "cores": 1, "kind": "port", "host": host,
                "sample": "main.cpp SmithWatermanScore restated (full (m+1)x(n+1)x3 int32 matrices, one contiguous "
                          "block instead of main.cpp's vector<vector<int>> rows: faster than the reference itself), "
                          "1 thread as in the reference, on row prefixes of the C2 pair up to %d x %d; %.1f s"
                          % (rows, len(a), t_tot)}
    if kind == "slab":
        # C5: main.cpp's full matrices would need 13.2 TB; lazySmith.cpp's linear-space
        # restatement on row prefixes of the C5 pair
        a, b = oracle.gen_pair(1048576 if n == 1 << 20 else n, n)
        rows, spent, cells, t_tot = 4, 0.0, 0, 0.0
        while True:
            t0 = time.perf_counter()
            oracle.score_linear(a, b, p, rows=rows)
            dt = time.perf_counter() - t0
            cells += rows * len(a); t_tot += dt; spent += dt
            if spent > budget_s or rows >= len(b):
                break
            rows = min(len(b), rows * 2)
        return {"value": cells / t_tot / 1e9, "unit": "GCUPS", "cores": 1, "kind": "port", "host": host,
                "sample": "lazySmith.cpp LazySmith restated (linear space; main.cpp's matrices need 13.2 TB), "
                          "1 thread, on row prefixes of the C5 pair up to %d x %d; %.1f s" % (rows, len(a), t_tot)}
    # batch: one pair per thread (embarrassingly parallel) on every core the job has
    npairs = threads
    pairs = [oracle.gen_pair(8192 + k, n) for k in range(npairs)]
    t0 = time.perf_counter()
    oracle.score_batch(pairs, p, threads=threads, full=True)
    dt = time.perf_counter() - t0
    # the same pairs in linear space (lazySmith.cpp LazySmith restated): the full-matrix figure above
    # runs every core against its own 805 MB matrices, so it is memory-bound; this one is the fair
    # all-core CPU rate
    t0 = time.perf_counter()
    oracle.score_batch(pairs, p, threads=threads, full=False)
    dl = time.perf_counter() - t0
    return {"value": npairs * n * n / dt / 1e9, "unit": "GCUPS", "cores": threads, "kind": "port", "host": host,
            "sample": "main.cpp SmithWatermanScore restated (full matrices), one pair per thread on all %d cores "
                      "of this job, %d pairs of %d x %d (seeds 8192+k); %.1f s" % (threads, npairs, n, n, dt),
            "linear_space": {"value": npairs * n * n / dl / 1e9, "unit": "GCUPS", "cores": threads,
                             "sample": "lazySmith.cpp LazySmith restated (two rows, linear space), the same %d pairs, "
                                       "one per thread; %.1f s" % (npairs, dl)}}


def profile_for(workload):
    """profiles/pmc_<workload>.json when it was taken with THIS library build."""
    import concurrentproject_amd as sw
    path = os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)
    if not os.path.exists(path):
        return None, "no profile"
    try:
        prof = json.load(open(path))
    except Exception as e:
        return None, repr(e)
    # the profile's kernels must be this build's: same library file, or (after a
    # rebuild) the same engine sources and flags
    if prof.get("lib_sha256") != lib_sha256(sw.LIB_PATH) and prof.get("source_sha256") != sw.source_stamp():
        return None, "stale: profile taken with another build of the engine"
    with open(path, "rb") as f:
        prof["_file_sha256"] = hashlib.sha256(f.read()).hexdigest()
    return prof, os.path.relpath(path, ROOT)


def issue_bound(prof, avg_kern_ms, waves_per_simd):
    """The kernel's VALU issue-time bound from the measured per-class issue costs
    (tools/issue_model.py, profiles/r03_ubench_issue_classes.jsonl): the profiled
    SQ_INSTS_VALU priced at the ns per SIMD of its chunk loop's instruction mix at this
    launch's waves per SIMD, spread over the 1024 SIMDs.  The guide's 2-cycle peak above
    holds for VOP1/VOP2-class instructions only; 3-source VOP3, VOP3P, DPP and SDWA
    forms issue at ~1.75-1.9 ns per SIMD however many waves share it."""
    mix = (prof or {}).get("valu_mix")
    if not mix or not prof.get("valu_insts_per_launch"):
        return None
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import issue_model
    table = issue_model.cost_table()
    ns = issue_model.issue_ns(mix["mix"], waves_per_simd, table)
    bound_ms = prof["valu_insts_per_launch"] * ns / (256 * 4) / 1e6
    return {"bound_ms": round(bound_ms, 4), "frac": round(bound_ms / avg_kern_ms, 4), "waves_per_simd": waves_per_simd,
            "ns_per_valu_per_simd": round(ns, 4), "mix": {k: round(v, 4) for k, v in mix["mix"].items()},
            "source": "tools/issue_model.py + profiles/r03_ubench_issue_classes.jsonl"}


def resident_waves_per_simd(st, torch):
    """Waves per SIMD of a launch: its workgroups' waves (4; the staged flow2 kernel 5)
    up to the occupancy the engine planned with (sw_last_stats waves_per_cu)."""
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    wpb = 5 if st["mode"] == 5 and not st["variant"] & 2 else 4
    waves = min(st["blocks"] * wpb, cus * max(1, st["waves_per_cu"]))
    return max(1, round(waves / (cus * 4)))


def roofline(workload, per_launch_cells, avg_kern_ms, step_ns=None, n=0, m=0, w2=False, waves_per_simd=None):
    prof, src = profile_for(workload)
    t = avg_kern_ms * 1e-3
    out = {"bound": "valu", "unit": "Tlane-ops/s", "peak": round(VALU_PEAK_TOPS, 2), "achieved": None, "frac": None,
           "traffic": None, "source": src}
    if prof is not None:
        # the exact profile file this line was computed from (tools/check_bench_lines.py)
        out["pmc_sha256"] = prof["_file_sha256"]
        out["lib_sha256"] = prof.get("lib_sha256")
    if prof is not None and prof.get("valu_insts_per_launch"):
        ops = prof["valu_insts_per_launch"] * 64
        out["achieved"] = round(ops / t / 1e12, 3)
        out["frac"] = round(ops / t / 1e12 / VALU_PEAK_TOPS, 4)
        out["valu_lane_ops_per_launch"] = ops
        out["valu_insts_per_cell"] = round(prof["valu_insts_per_launch"] * 64 / per_launch_cells, 3)
    if prof is not None and waves_per_simd:
        out["issue"] = issue_bound(prof, avg_kern_ms, waves_per_simd)
    if prof is not None:
        out["traffic"] = prof.get("hbm_bytes_per_launch")
        if prof.get("clock_ghz"):
            out["profiled_clock_ghz"] = prof["clock_ghz"]
    algo = per_launch_cells * ALGO_BYTES_PER_CELL
    out["hbm"] = {"algorithmic_bytes_per_launch": algo,
                  "algorithmic_frac": round(algo / t / 1e9 / HBM_PEAK_GBS, 4),
                  "traffic_frac": (round(out["traffic"] / t / 1e9 / HBM_PEAK_GBS, 4) if out["traffic"] else None),
                  "note": "12 B/cell (int32 H, E, F, SURVEY 8d) is notional: the kernel keeps them on chip, so "
                          "algorithmic_frac can exceed 1; traffic_frac is the counted HBM bytes"}
    if step_ns:
        # the wavefront's own bound at the measured step: strip s can start its row i no
        # sooner than 63 steps after strip s-1 did (the lane skew), so the last strip ends
        # after m + 63 * strips steps (W = 1: ~ n + m; two columns per lane: ~ m + n / 2)
        strips = flow2_strips(n, w2)
        out["step_ns"] = round(step_ns, 3)
        out["wavefront_steps"] = m + 63 * strips
        out["critical_path_frac"] = round((m + 63 * strips) * step_ns / (avg_kern_ms * 1e6), 4)
        # the same path at the lone-wave issue time of the bare two-column step body (no
        # hand-offs, no chunk work: tools/ubench_w2seq.hip, 4 steps of the compiled W2 loop)
        body = os.path.join(ROOT, "profiles", "r03_ubench_w2_step_body.jsonl")
        if w2 and os.path.exists(body):
            rows = [json.loads(l) for l in open(body) if l.startswith("{")]
            body_ns = min(r["ns_per_4steps"] for r in rows) / 4
            out["step_body_ns"] = round(body_ns, 3)
            out["issue_path_frac"] = round((m + 63 * strips) * body_ns / (avg_kern_ms * 1e6), 4)
    return out


def kernel_label(st):
    """What a launch ran, from sw_last_stats (mode + variant bits, sw_engine.hip enqueue):
    the kernel family, the HIP function it launched (the name rocprof reports), the columns
    per lane actually computed and the step (the exact linear-gap identity at G_INIT ==
    G_EXT, DESIGN.md section 2, or the general affine Gotoh step)."""
    v, mode = st["variant"], st["mode"]
    lin = bool(v & 8)
    out = {"W": st["W"]}
    if mode == 5:
        ring, w2, f3, hl, aff3 = bool(v & 4), bool(v & 16), bool(v & 64), bool(v & 512), bool(v & 1024)
        if f3 or aff3:
            name = ("flow3 ring" if ring else "flow3") + (" affine" if aff3 else "") + (" W3" if v & 8192 else "") + \
                (" W4/W5" if v & 16384 else "") + (" pool loops" if v & 4096 else "")
            if v & 32768:
                name = "flow3 W3%s, pair per workgroup" % (" affine" if aff3 else "")
            fn = "sw_flow3p_kernel" if v & 4096 else "sw_flow3r45_kernel" if v & 16384 else \
                ("sw_flow3ra3p_kernel" if aff3 else "sw_flow3r3p_kernel") if v & 32768 else \
                ("sw_flow3r" if ring else "sw_flow3") + ("a" if aff3 else "") + ("3" if v & 8192 else "") + \
                ("s" if v & 2048 else "") + "_kernel"
            if v & 65536:   # a pair over up to seven byte values (sw_flow3h / sw_flow3ah_kernel)
                name += ", seven-letter alphabet"
                fn = ("sw_flow3r%s3h_kernel" % ("a" if aff3 else "")) if ring else \
                    "sw_flow3ah_kernel" if aff3 else "sw_flow3h_kernel"
            if v & 2048:
                name += ", column slab (peer edges)"
        else:
            name = "flow2 " + ("pair per workgroup" if v & 32 else "ring" if ring else "streamed" if v & 2 else "staged")
            fn = "sw_flow2_kernel"
        if hl:
            name += ", half-chunk links"
        out["W"] = 4 if v & 16384 else 3 if v & 8192 else 2 if w2 else 1
    elif mode == 3:
        name = "duo" + (" LDS hand-offs" if v & 128 else " granules") + (", row-code table" if v & 256 else "") + \
               (", f16-max3" if v & 1 else "")
        fn = "sw_duo_lds_kernel" if v & 128 else "sw_duo_kernel"
        if st.get("dna") == 0:
            name += ", raw bytes"
        lin = bool(v & 8)
    else:
        name = {0: "strip", 1: "pairwg", 2: "chain", 4: "flow"}.get(mode, str(mode))
        fn = {0: "sw_strip_kernel", 1: "sw_pairwg_kernel", 2: "sw_chain_kernel", 4: "sw_flow_kernel"}.get(mode, "?")
    out.update(kernel=name, kernel_fn=fn, C=st["C"],
               step="linear-gap identity (G_INIT == G_EXT, exact)" if lin else "affine (Gotoh E/F)")
    return out


AFFINE_PARAMS = (2, -3, 5, 2)   # G_INIT != G_EXT: the general Gotoh step (goldens C2_affine, C3_affine, C5_affine)


def affine_runs(sw, torch, launch, scores, stream, gold, N, steps, params, defaults):
    """N = 1 extras of the pair workload: the general affine step (G_INIT != G_EXT, params
    AFFINE_PARAMS) on the C2 pair against its reference-pinned golden, and the same step
    forced at the default constants (option linear = 0: no linear-gap identity)."""
    out = {}
    st_steps = max(3, steps // 2)
    try:
        sw.set_params(sw.Params(*AFFINE_PARAMS))
        at, ak = time_launches(torch, launch, lambda: None, st_steps, 1, stream, None)
        sw.stream_status(stream.cuda_stream)
        st = sw.last_stats()
        g = gold.get("C2_affine", {})
        out = {"params": list(AFFINE_PARAMS), "ms_per_step": round(at / st_steps * 1e3, 4),
               "value": round(N * N * st_steps / at / 1e9, 3), "unit": "GCUPS",
               "kernel_ms_per_launch": round(ak, 4), "kernel_gcups": round(N * N / (ak * 1e-3) / 1e9, 3),
               "parity": ("ok" if scores[0].item() == g["score"] else "MISMATCH") if g and N == 65536 else "unchecked",
               "golden": "C2_affine (reference LazySmith built with these constants)", **kernel_label(st),
               "roofline": roofline("pair_affine", N * N, ak)}
    finally:
        sw.set_params(sw.Params(*params))
    sw.set_option("linear", 0)
    try:
        at, ak = time_launches(torch, launch, lambda: None, st_steps, 1, stream, None)
        sw.stream_status(stream.cuda_stream)
        ok = ("ok" if scores[0].item() == gold.get("C2", {}).get("score") else "MISMATCH") \
            if defaults and N == 65536 else "unchecked"
        out["default_consts_linear0"] = {"kernel_ms_per_launch": round(ak, 4),
                                         "kernel_gcups": round(N * N / (ak * 1e-3) / 1e9, 3), "parity": ok,
                                         **kernel_label(sw.last_stats()),
                                         "note": "option linear=0: the affine step at (1,-1,1,1) on the C2 pair"}
    finally:
        sw.set_option("linear", -1)
    return out


def batch_affine_runs(sw, torch, gold, steps, params, cells):
    """N = 1 extras of the batched workload: C3 (1024 pairs N = 8192, seeds 8192 + k) with the
    general Gotoh step at AFFINE_PARAMS, on the automatic plan (the packed-u16 duo kernel) and on
    the int32 pair-per-workgroup kernel, each against the reference-pinned golden C3_affine."""
    ref = gold.get("C3_affine", {}).get("scores", [])
    out = {}
    sw.set_params(sw.Params(*AFFINE_PARAMS))
    try:
        bt, bk, bsc, bcells, bst = run_batch(sw, torch, None, 1, 0, 8192, 1024, steps, 1)
        out = {"params": list(AFFINE_PARAMS), "workload": "C3 batch of 1024 pairs N=8192 (seeds 8192+k)",
               "value": round(bcells * steps / bt / 1e9, 3), "unit": "GCUPS",
               "ms_per_step": round(bt / steps * 1e3, 4), "kernel_ms_per_launch": round(bk, 4),
               "kernel_gcups": round(bcells / (bk * 1e-3) / 1e9, 3),
               "parity": ("ok" if bsc == ref else "MISMATCH") if len(ref) == 1024 else "unchecked",
               "golden": "C3_affine (all 1024 pairs, reference LazySmith built with these constants)",
               **kernel_label(bst),
               "dtype": "u16x2 (packed, exact: scores < 2^16)" if bst["mode"] == 3 else "int32",
               "roofline": roofline("batch" + affine_key(bst), bcells, bk,
                                    waves_per_simd=resident_waves_per_simd(bst, torch))}
        sw.set_option("mode", 5)
        sw.set_option("f2pwg", 1)
        try:
            it, ik, isc, _, ist = run_batch(sw, torch, None, 1, 0, 8192, 1024, 2, 1)
            out["int32_kernel"] = {"kernel_ms_per_launch": round(ik, 4),
                                   "kernel_gcups": round(bcells / (ik * 1e-3) / 1e9, 3),
                                   "parity": ("ok" if isc == ref else "MISMATCH") if len(ref) == 1024 else "unchecked",
                                   **kernel_label(ist)}
        finally:
            sw.set_option("mode", -1)
            sw.set_option("f2pwg", -1)
    finally:
        sw.set_params(sw.Params(*params))
    return out


def alphabet_runs(sw, torch, gold, steps):
    """N = 1 extras: the config pairs with their bases relabeled to lower case (a, c, g, t: bytes
    outside {A,C,G,T}, a bijection, so the reference scores and the goldens are unchanged; main.cpp
    scores by byte equality).  C2 and C5 then take the seven-letter kernels (one pair, the alphabet
    scanned on the device each call: sw_flow3h_kernel / sw_flow3r3h_kernel), C3 the duo kernel with
    the penalty from the raw bytes (SW_FLAG_BYTES, no scan); each against its golden."""
    lower = np.arange(256, dtype=np.uint8)
    for ch in b"ACGT":
        lower[ch] = ch + 32
    out = {"relabel": "A,C,G,T -> a,c,g,t (bytes outside {A,C,G,T}; goldens unchanged)"}
    stream = torch.cuda.current_stream()
    for key, N, seed, gk, nsteps in (("c2_lower", 65536, 65536, "C2", steps), ("c5_lower", 1 << 20, 1 << 20, "C5", 2)):
        a, b = sw.gen_pair(seed, N)
        arena = torch.from_numpy(np.concatenate([lower[a], lower[b]])).cuda()
        scores = torch.zeros(1, dtype=torch.int32, device="cuda")

        def launch():
            sw.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], scores.data_ptr(), flags=0,
                                  stream=stream.cuda_stream)
        t, k = time_launches(torch, launch, lambda: None, nsteps, 1, stream, None)
        sw.stream_status(stream.cuda_stream)
        st = sw.last_stats()
        g = gold.get(gk, {})
        out[key] = {"N": N, "ms_per_step": round(t / nsteps * 1e3, 4), "value": round(N * N * nsteps / t / 1e9, 3),
                    "unit": "GCUPS", "kernel_ms_per_launch": round(k, 4), "steps": nsteps,
                    "parity": ("ok" if scores[0].item() == g["score"] else "MISMATCH") if g else "unchecked",
                    "golden": gk, "alphabet": "seven-letter path" if st["dna"] == 2 else "dna %d" % st["dna"],
                    "timed": "device entry incl. the alphabet scan and its host sync per call", **kernel_label(st)}
    host = lower[sw.gen_batch(8192, 1024, 8192)]
    arena = torch.from_numpy(host).cuda()
    scores = torch.zeros(1024, dtype=torch.int32, device="cuda")
    offs_a = [2 * 8192 * k for k in range(1024)]
    offs_b = [2 * 8192 * k + 8192 for k in range(1024)]

    def launch_b():
        sw.score_batch_device(arena.data_ptr(), offs_a, [8192] * 1024, offs_b, [8192] * 1024, scores.data_ptr(),
                              flags=sw.SW_FLAG_BYTES, stream=stream.cuda_stream)
    bsteps = max(3, steps // 2)
    t, k = time_launches(torch, launch_b, lambda: None, bsteps, 1, stream, None)
    sw.stream_status(stream.cuda_stream)
    st = sw.last_stats()
    ref = gold.get("C3", {}).get("scores", [])
    cells = 1024 * 8192 * 8192
    out["c3_lower"] = {"ms_per_step": round(t / bsteps * 1e3, 4), "value": round(cells * bsteps / t / 1e9, 3),
                       "unit": "GCUPS", "kernel_ms_per_launch": round(k, 4), "steps": bsteps,
                       "parity": ("ok" if scores.cpu().tolist() == ref else "MISMATCH") if len(ref) == 1024 else "unchecked",
                       "golden": "C3 (all 1024 pairs)", "alphabet": "raw bytes" if st["dna"] == 0 else "dna %d" % st["dna"],
                       **kernel_label(st)}
    return out


def c5_runs(sw, torch, gold, steps):
    """N = 1 extras: config C5 (one pair N = 2^20, seed 1048576, O(N) device state) with the
    reference's constants and with AFFINE_PARAMS, each against its golden."""
    N = 1 << 20
    a, b = sw.gen_pair(1048576, N)
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    scores = torch.zeros(1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def launch():
        sw.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], scores.data_ptr(), flags=1,
                              stream=stream.cuda_stream)
    out = {}
    for key, prm, gk in (("linear", (1, -1, 1, 1), "C5"), ("affine", AFFINE_PARAMS, "C5_affine")):
        sw.set_params(sw.Params(*prm))
        try:
            t, k = time_launches(torch, launch, lambda: None, steps, 1, stream, None)
            sw.stream_status(stream.cuda_stream)
            g = gold.get(gk, {})
            out[key] = {"params": list(prm), "ms_per_step": round(t / steps * 1e3, 3),
                        "value": round(N * N * steps / t / 1e9, 3), "unit": "GCUPS",
                        "kernel_ms_per_launch": round(k, 3), "steps": steps,
                        "parity": ("ok" if scores[0].item() == g["score"] else "MISMATCH") if g else "unchecked",
                        "score": scores[0].item(), **kernel_label(sw.last_stats()),
                        "boundary_bytes": sw.last_stats()["boundary_bytes"],
                        "roofline": roofline("slab" if key == "linear" else "slab_affine", N * N, k,
                                             waves_per_simd=resident_waves_per_simd(sw.last_stats(), torch))}
        finally:
            sw.set_params(sw.Params(1, -1, 1, 1))
    out["workload"] = "C5 single pair N=2^20 (seed 1048576), resident in HBM"
    return out


def headline_summary(out):
    """{workload: [ms_per_step, GCUPS, parity]} of the line's main workload and its nested extras."""
    def row(d):
        return [d.get("ms_per_step"), round(d["value"]) if d.get("value") is not None else None, d.get("parity")]
    wl = (out.get("config") or {}).get("workload", "main")
    key = "c2" if wl.startswith("C2") else "c3" if wl.startswith("C3") else "c4" if wl.startswith("C4") else \
        "c5" if wl.startswith("C5") else "main"
    if out.get("config", {}).get("params") == list(AFFINE_PARAMS):
        key += "_affine"
    res = {key: row(out)}
    if isinstance(out.get("affine_step"), dict) and out["affine_step"].get("value") is not None:
        res["c2_affine"] = row(out["affine_step"])
    b = out.get("batch_c3") or out.get("batch_c4")
    if isinstance(b, dict):
        res["c3" if "batch_c3" in out else "c4"] = row(b)
        if isinstance(b.get("affine_step"), dict) and b["affine_step"].get("value") is not None:
            res["c3_affine"] = row(b["affine_step"])
        if isinstance(b.get("int32_kernel"), dict):
            res["c3_int32_kernel_ms"] = b["int32_kernel"].get("kernel_ms_per_launch")
    for k in ("linear", "affine"):
        c = (out.get("c5") or {}).get(k)
        if isinstance(c, dict):
            res["c5" if k == "linear" else "c5_affine"] = row(c)
    for k, c in (out.get("byte_alphabets") or {}).items():
        if isinstance(c, dict):
            res[k] = row(c)
    res["units"] = "[ms_per_step, GCUPS, parity]"
    return res


def affine_key(st):
    """"_affine" when a launch ran the general affine step (its counter profile is
    profiles/pmc_<workload>_affine.json, tools/pmc_summary.py c2a / c3a / c5a)."""
    return "_affine" if st["mode"] in (3, 5) and not st["variant"] & 8 else ""


def flow2_strips(n, w2=False):
    """Strips of the single-pair kernel (sw_internal.h flow2_strips / flow2_strips_w2)."""
    if w2:
        return 1 if n <= 128 else (n - 2 + 125) // 126
    return 1 if n <= 64 else (n - 1 + 62) // 63


def measure_step_ns(sw, torch, arena, offs_a, lens, offs_b, scores, sptr, N):
    """Step time of the single-pair kernel's first strip (no inflow: its own pace)
    from one traced launch: (end - start) / (m + 63) steps, s_memrealtime 100 MHz."""
    st = sw.last_stats()
    if st["mode"] != 5:
        return None
    strips = flow2_strips(N, bool(st["variant"] & 16))
    trace = torch.zeros(16 * strips, dtype=torch.int64, device="cuda")
    sw.set_option("trace", trace.data_ptr())
    try:
        sw.score_batch_device(arena.data_ptr(), offs_a, lens, offs_b, lens, scores.data_ptr(), flags=1, stream=sptr)
        torch.cuda.synchronize()
    finally:
        sw.set_option("trace", 0)
    sw.stream_status(sptr)
    t = trace.cpu().numpy().reshape(strips, 16)
    return float(t[0, 2] - t[0, 0]) * 10.0 / (N + 63)


def time_launches(torch, launch, collective, steps, warmup, stream, dist):
    """Time `steps` launches (+ their collective) between barrier + synchronize brackets;
    returns (max-over-ranks wall seconds, mean kernel ms from HIP events on `stream`).
    stream None (CPU ranks of the tests): wall time only, kernel ms None."""
    gpu = stream is not None
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    for _ in range(warmup):
        launch()
        collective()
    sync()
    starts = [torch.cuda.Event(enable_timing=True) for _ in range(steps)] if gpu else []
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(steps)] if gpu else []
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        if gpu:
            starts[i].record(stream)
        launch()
        if gpu:
            ends[i].record(stream)
        collective()
    sync()
    if dist is not None:
        dist.barrier()
    t_local = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in zip(starts, ends)])) if gpu else None
    t_max = t_local
    if dist is not None:
        tt = torch.tensor([t_local], dtype=torch.float64, device="cuda" if gpu else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
    return t_max, kern_ms


class BatchRank:
    """One rank's share of the batched workload (C3 at one GPU, C4 at eight): the
    contiguous block shard_bounds(P * world, world, rank) of the global batch (pair k
    seeded 8192 + k, N x N), scored with no data-path collective; `collective` gathers
    the int32 scores to rank 0 (RCCL; gloo in the CPU tests).
    scorer "engine": the HIP kernels on the sequences resident in HBM (sw_score_batch_device);
    "oracle": the CPU restatement (tests/launch_worker.py runs this class on gloo ranks)."""

    def __init__(self, torch, dist, world, rank, N, P, scorer="engine"):
        from concurrentproject_amd.dist import shard_bounds
        self.torch, self.dist, self.world, self.P = torch, dist, world, P
        self.lo, self.hi = shard_bounds(P * world, world, rank)
        self.npairs = npairs = self.hi - self.lo
        self.cells = npairs * N * N
        self.gathered = None
        if scorer == "engine":
            import concurrentproject_amd as sw
            host = sw.gen_batch(8192 + self.lo, npairs, N)
            self.arena = torch.from_numpy(host).cuda()
            self.scores = torch.zeros(npairs, dtype=torch.int32, device="cuda")
            self.stream = torch.cuda.current_stream()
            offs_a = [2 * N * k for k in range(npairs)]
            offs_b = [2 * N * k + N for k in range(npairs)]

            def launch():
                sw.score_batch_device(self.arena.data_ptr(), offs_a, [N] * npairs, offs_b, [N] * npairs,
                                      self.scores.data_ptr(), flags=1, stream=self.stream.cuda_stream)
            self.launch = launch
        else:
            import oracle
            pairs = [oracle.gen_pair(8192 + k, N) for k in range(self.lo, self.hi)]
            self.scores = torch.zeros(npairs, dtype=torch.int32)
            self.stream = None
            self.launch = lambda: self.scores.copy_(torch.tensor(oracle.score_batch(pairs), dtype=torch.int32))

    def collective(self):
        if self.dist is not None:
            from concurrentproject_amd.dist import gather_scores
            self.gathered = gather_scores(self.scores, self.P * self.world)

    def result(self):
        """Rank 0: every pair's score in global order (a rank without a group: its own)."""
        if self.gathered is not None:
            return self.gathered.cpu().tolist()
        return self.scores.cpu().tolist() if self.dist is None else None


def run_batch(sw, torch, dist, world, rank, N, P, steps, warmup):
    """C3 (one GPU) / C4 (sharded): BatchRank timed over `steps` launches."""
    job = BatchRank(torch, dist, world, rank, N, P)
    t_max, kern_ms = time_launches(torch, job.launch, job.collective, steps, warmup, job.stream, dist)
    sw.stream_status(job.stream.cuda_stream)
    return t_max, kern_ms, job.result(), job.cells, sw.last_stats()


class OracleSlabs:
    """The CPU stand-in of dist.ColumnSlabs in the gloo tests: the same bounds
    (sw_slab_bounds), the same all-reduce(MAX) of one int, with the edge column
    passed rank to rank by gloo send/recv in place of the kernel's IPC stores."""

    def __init__(self, dist, n, m, a, b):
        import concurrentproject_amd as sw
        self.dist, self.n, self.m, self.a, self.b = dist, n, m, a, b
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.bounds = sw.slab_bounds(n, m, self.world, sw.SW_FLAG_DNA)
        self.inflow = None

    @property
    def columns(self):
        return self.bounds[self.rank], self.bounds[self.rank + 1]

    def launch(self):
        import oracle
        import torch
        lo, hi = self.columns
        edge = None
        if self.rank > 0:
            eh, ee = torch.empty(self.m, dtype=torch.int32), torch.empty(self.m, dtype=torch.int32)
            self.dist.recv(eh, src=self.rank - 1)
            self.dist.recv(ee, src=self.rank - 1)
            edge = (eh.numpy(), ee.numpy())
        best, (oh, oe) = oracle.slab(self.a[lo:hi], self.b, edge=edge)
        if self.rank + 1 < self.world:
            self.dist.send(torch.from_numpy(np.ascontiguousarray(oh)), dst=self.rank + 1)
            self.dist.send(torch.from_numpy(np.ascontiguousarray(oe)), dst=self.rank + 1)
        self.score = torch.tensor([best], dtype=torch.int32)

    def reduce(self):
        from concurrentproject_amd.dist import slab_max
        return slab_max(self.score)

    def close(self):
        pass


class SlabRank:
    """One rank's slab of the C5 pair cut into column slabs (f-1): `launch` scores it
    (dist.ColumnSlabs: the kernel stores its right edge into the next rank's IPC-mapped
    fine-grained buffer, and the all-reduce(MAX) of the slab maxima follows on the same
    stream); `report` gathers the per-rank kernel times, columns, pipeline fill and
    inflow memory kinds.  scorer "oracle": OracleSlabs on gloo (tests)."""

    def __init__(self, torch, dist, n, m, a, b, scorer="engine"):
        self.torch, self.dist = torch, dist
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.score = None
        if scorer == "engine":
            import concurrentproject_amd as sw
            from concurrentproject_amd.dist import ColumnSlabs
            self.arena = torch.from_numpy(np.concatenate([a, b])).cuda()
            self.slabs = ColumnSlabs(n, m, sw.SW_FLAG_DNA)
            self.stream = torch.cuda.current_stream()
            self.launch = lambda: self.slabs.launch(self.arena.data_ptr(), 0, n, self.stream.cuda_stream)
        else:
            self.slabs = OracleSlabs(dist, n, m, a, b)
            self.stream = None
            self.launch = self.slabs.launch
        inflow = self.slabs.inflow
        self.fine_grained = inflow.fine_grained if inflow is not None else None
        lo, hi = self.slabs.columns
        self.cells = (hi - lo) * m

    def collective(self):
        """The all-reduce(MAX) of the slab maxima (RCCL; after the kernel's event, so the
        per-rank kernel times keep the pipeline fill)."""
        self.score = self.slabs.reduce()

    def report(self, kern_ms):
        """Every rank's launch-to-end kernel time (rank r's includes its wait for rank r-1's
        first edge rows: last - first is the pipeline fill), columns and inflow memory kind."""
        torch, dist, world = self.torch, self.dist, self.world
        kind = {None: -1.0, True: 1.0, False: 0.0}[self.fine_grained]
        kt = torch.tensor([kern_ms if kern_ms is not None else -1.0, kind], dtype=torch.float64,
                          device="cuda" if self.stream is not None else "cpu")
        allk = [torch.zeros_like(kt) for _ in range(world)]
        dist.all_gather(allk, kt)
        per_rank = [round(float(x[0].item()), 4) for x in allk]
        b = self.slabs.bounds
        return {"per_rank_kernel_ms": per_rank, "per_rank_columns": [b[r + 1] - b[r] for r in range(world)],
                "pipeline_fill_ms": round(per_rank[-1] - per_rank[0], 4),
                "inflow_fine_grained": [{1.0: True, 0.0: False}.get(float(x[1].item())) for x in allk],
                "note": "rank 0 runs at its own pace; rank r's kernel also waits for the first edge rows of rank "
                        "r-1, so last - first is the fill of the R-1 hops; inflow_fine_grained: each rank's inflow "
                        "buffer (rank 0 has none; an edge written by another GPU needs fine-grained memory)"}

    def result(self):
        return int(self.score[0].item())

    def close(self):
        self.slabs.close()


def start_ranks(args) -> int | None:
    """Standalone `--gpus N` (N > 1, no launcher variables): check the devices and run
    N ranks of this script (concurrentproject_amd.launch.spawn_ranks); returns the
    job's exit status.  None when this process is to run as a rank itself.  Nothing
    here initialises the GPU (device_count only), and the ranks are child processes."""
    from concurrentproject_amd.launch import LaunchError, launcher_env, require_devices, spawn_ranks
    if launcher_env() or (args.gpus or 1) <= 1:
        return None
    try:
        require_devices(args.gpus)
    except LaunchError as e:
        print("bench.py: %s" % e, file=sys.stderr, flush=True)
        return 2
    return spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:])


def main():
    args = parse()
    status = start_ranks(args)
    if status is not None:
        sys.exit(status)
    from concurrentproject_amd.launch import launcher_env, rank_env, visible_devices
    world, rank, local = rank_env()
    if args.gpus is not None and args.gpus != world:
        sys.exit("bench.py: --gpus %d but the launcher started %d ranks (WORLD_SIZE)" % (args.gpus, world))
    if local >= visible_devices():
        sys.exit("bench.py: rank %d needs GPU %d, this host shows %d" % (rank, local, visible_devices()))
    import torch
    torch.cuda.set_device(local)
    # launches go on a stream of their own: on torch's default stream cuda_stream is 0, and
    # sw_score_batch_device then runs its blocking form (a stream sync and error check per call,
    # the GPU idle while the host plans the next one: 0.35 ms a C3 step, profiles/r05_c3_hip_trace.md)
    torch.cuda.set_stream(torch.cuda.Stream())
    dist = None
    rccl = None
    if world > 1 or launcher_env():
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world, rank = dist.get_world_size(), dist.get_rank()
        rccl = {"backend": dist.get_backend(), "world_size": world}
    import concurrentproject_amd as sw
    params = tuple(int(x) for x in args.params.split(","))
    sw.set_params(sw.Params(*params))
    if args.W:
        sw.set_option("W", args.W)
    if args.C:
        sw.set_option("C", args.C)
    if args.mode >= 0:
        sw.set_option("mode", args.mode)
    for kv in args.opt:
        k, v = kv.split("=")
        sw.set_option(k, int(v))
    gold = load_golden()
    defaults = params == (1, -1, 1, 1)

    workload = args.workload
    if workload == "auto":
        workload = "pair"     # the same per-GPU work at every N (module docstring)
    slab_ranks = None

    extra = None
    c5 = None
    alpha = None
    affine = None
    step_ns = None
    host_api = None
    parity = "unchecked"
    if workload == "batch":
        N = args.n or 8192
        P = args.pairs_per_gpu
        t_max, avg_kern_ms, allsc, cells_rank, st = run_batch(sw, torch, dist, world, rank, N, P, args.steps,
                                                              args.warmup)
        cells_job = cells_rank * world
        per_launch_cells = cells_rank
        cfg = {"workload": ("C4 batch, %d pairs/GPU (%d pairs)" % (P, P * world)) if world > 1
               else "C3 batch of %d pairs" % P, "N": N, "pairs_per_gpu": P, "global_pairs": P * world,
               "parallelism": "pair-sharded x%d + RCCL gather of scores" % world if world > 1 else "single GPU"}
        if rank == 0 and defaults and N == 8192:
            ref = gold.get("C4", gold.get("C3", {})).get("scores", [])
            if len(ref) >= len(allsc):
                parity = "ok" if allsc == ref[:len(allsc)] else "MISMATCH"
        elif rank == 0 and params == AFFINE_PARAMS and N == 8192 and world == 1:
            ref = gold.get("C3_affine", {}).get("scores", [])
            if len(ref) == len(allsc):
                parity = "ok" if allsc == ref else "MISMATCH"
    else:
        slabs, slab_buf, slab_cols = None, None, None
        if workload == "pair":
            # C2 at N=1; at N GPUs a global batch of N such pairs (pair k seeded 65536+k)
            N = args.n or 65536
            a, b = sw.gen_pair(65536 + rank, N)
            cfg = {"workload": "C2 single pair N=%d (seed 65536)" % N if world == 1 else
                               "C2-size pairs N=%d, one per GPU (seeds 65536+rank)" % N,
                   "N": N, "pairs_per_gpu": 1, "global_pairs": world,
                   "parallelism": "pair-sharded x%d + RCCL gather of scores" % world if world > 1 else "single GPU"}
        else:
            # C5: ONE pair N = 2^20 (seed 1048576); every rank holds the whole pair (2 MB)
            N = args.n or (1 << 20)
            a, b = sw.gen_pair(1048576 if N == 1 << 20 else N, N)
            cfg = {"workload": "C5 single pair N=%d (seed 1048576)" % N, "N": N, "pairs_per_gpu": 1.0 / world,
                   "global_pairs": 1,
                   "parallelism": ("column slabs x%d, GPU-to-GPU edge stores + RCCL all-reduce(MAX)" % world
                                   if world > 1 else "single GPU")}
        host = np.concatenate([a, b])
        arena = torch.from_numpy(host).cuda()
        scores = torch.zeros(1, dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream()
        sptr = stream.cuda_stream
        offs_a, offs_b, lens = [0], [N], [N]
        cells_rank = cells_job = N * N
        if workload == "slab" and dist is not None:
            slabs = SlabRank(torch, dist, N, N, a, b)
            lo, hi = slabs.slabs.columns
            cells_rank, cells_job = slabs.cells, N * N
            cfg["slab_columns"] = [lo, hi]
        elif workload == "slab" and args.slab_of > 1:
            bounds = sw.slab_bounds(N, N, args.slab_of, sw.SW_FLAG_DNA)
            slab_cols, slab_buf = bounds[1], sw.slab_alloc(N)
            cells_rank = cells_job = slab_cols * N
            cfg.update(workload="C5 slab 0 of a %d-way column split, alone (per-rank cost)" % args.slab_of,
                       slab_columns=[0, slab_cols])
        elif workload == "pair":
            cells_job = N * N * world
        per_launch_cells = cells_rank
        epoch = [0]
        gathered = [None]

        def launch():
            if slabs is not None:
                slabs.launch()
            elif slab_buf is not None:
                epoch[0] += 1
                sw.score_slab_device(arena.data_ptr(), 0, slab_cols, N, N, 0, slab_buf.ptr, epoch[0],
                                     scores.data_ptr(), sw.SW_FLAG_DNA, sptr)
            else:
                sw.score_batch_device(arena.data_ptr(), offs_a, lens, offs_b, lens, scores.data_ptr(),
                                      flags=1, stream=sptr)

        def collective():
            if dist is None:
                return
            if slabs is not None:
                slabs.collective()                         # RCCL all-reduce(MAX) of one int
            else:
                from concurrentproject_amd.dist import gather_scores
                gathered[0] = gather_scores(scores, world)  # RCCL gather of the per-pair int32 scores

        t_max, avg_kern_ms = time_launches(torch, launch, collective, args.steps, args.warmup, stream, dist)
        sw.stream_status(sptr)
        st = sw.last_stats()
        first = gathered[0][0].item() if gathered[0] is not None else scores[0].item()
        if slabs is not None:
            first = slabs.result()
            slab_ranks = slabs.report(avg_kern_ms)
            slabs.close()
        if slab_buf is not None:
            slab_buf.free()
        if rank == 0 and world == 1 and slab_buf is None:
            step_ns = measure_step_ns(sw, torch, arena, offs_a, lens, offs_b, scores, sptr, N)
        # PCIe-inclusive rate of the synchronous host entry point (H2D of the two
        # sequences + launch + score D2H): reported beside `value`, never as it
        if rank == 0 and workload == "pair":
            a_h, b_h = host[:N], host[N:]
            sw.SmithWatermanScoreCUDA(a_h, b_h)
            calls = 10
            t1 = time.perf_counter()
            hs = [sw.SmithWatermanScoreCUDA(a_h, b_h) for _ in range(calls)]
            dt = (time.perf_counter() - t1) / calls
            host_api = {"gcups": round(N * N / dt / 1e9, 3), "ms_per_call": round(dt * 1e3, 4), "calls": calls,
                        "score": hs[0], "scores_equal": len(set(hs)) == 1,
                        "entry": "SmithWatermanScoreCUDA (algoGPU.h:9), host buffers: H2D of both sequences, "
                                 "launch, score D2H, synchronous; mean of %d calls" % calls}
        # the goldens of the reference's constants (C2, C5) and of AFFINE_PARAMS (C2_affine, C5_affine)
        gkey = None
        if rank == 0 and (defaults or params == AFFINE_PARAMS):
            suffix = "" if defaults else "_affine"
            if workload == "pair" and N == 65536:   # rank 0's pair is the C2 pair
                gkey = "C2" + suffix
            elif workload == "slab" and N == 1 << 20 and slab_buf is None:
                gkey = "C5" + suffix
        if gkey is not None and gkey in gold:
            parity = "ok" if first == gold[gkey]["score"] else "MISMATCH"
        # N=1: the general affine step on the same pair (the automatic plan takes the
        # exact linear-gap step at G_INIT == G_EXT), for reference
        affine = None
        if workload == "pair" and world == 1 and args.workload == "auto" and not args.no_extra and \
                params[2] == params[3]:
            affine = affine_runs(sw, torch, launch, scores, stream, gold, N, args.steps, params, defaults)
        c5 = None
        if workload == "pair" and world == 1 and args.workload == "auto" and not args.no_extra and \
                not args.no_c5 and defaults and N == 65536:
            c5 = c5_runs(sw, torch, gold, 2)
        alpha = None
        if workload == "pair" and world == 1 and args.workload == "auto" and not args.no_extra and \
                not args.no_c5 and defaults and N == 65536:
            alpha = alphabet_runs(sw, torch, gold, args.steps)
        # the batched config measured right after on the same ranks, as an extra key:
        # C3 at N=1, 1024 pairs per GPU sharded + RCCL-gathered at N>1 (C4 at N=8)
        if workload == "pair" and args.workload == "auto" and not args.no_extra:
            bsteps = max(3, args.steps // 2)
            bt, bk, bsc, bcells, bst = run_batch(sw, torch, dist, world, rank, 8192, 1024, bsteps, 1)
            ref = gold.get("C4", gold.get("C3", {})).get("scores", [])
            extra = {"workload": ("C3 batch of 1024 pairs N=8192 (seeds 8192+k)" if world == 1 else
                                  "C4-order batch: %d pairs N=8192, 1024 per GPU (seeds 8192+k), RCCL gather"
                                  % (1024 * world)),
                     "n_gpus": world, "value": round(bcells * world * bsteps / bt / 1e9, 3),
                     "unit": "GCUPS", "ms_per_step": round(bt / bsteps * 1e3, 4), "kernel_ms_per_launch": round(bk, 4),
                     "kernel_gcups": round(bcells / (bk * 1e-3) / 1e9, 3),
                     "parity": ("ok" if bsc == ref[:len(bsc)] else "MISMATCH")
                     if defaults and len(ref) >= len(bsc) == 1024 * world else "unchecked",
                     **kernel_label(bst),
                     "dtype": "u16x2 (packed, exact: scores < 2^16)" if bst["mode"] == 3 else "int32",
                     "roofline": roofline("batch", bcells, bk, waves_per_simd=resident_waves_per_simd(bst, torch))}
        if extra is not None and world == 1:
            # the same batch on the int32 kernels (no 16-bit packing): the flow2 step with a
            # pair per workgroup, which the engine picks for batches whose scores need int32,
            # and the pair-per-workgroup strip kernel it replaced there
            for key, mode, pwg, f3pwg, name in (("int32_kernel", 5, 1, 1, "flow3 W3 pair per workgroup"),
                                                ("int32_flow2_kernel", 5, 1, 0, "flow2 pair per workgroup"),
                                                ("pairwg_kernel", 1, -1, 1, "pairwg")):
                sw.set_option("mode", mode)
                sw.set_option("f2pwg", pwg)
                sw.set_option("f3pwg", f3pwg)
                try:
                    it, ik, isc, _, ist = run_batch(sw, torch, None, 1, 0, 8192, 1024, 2, 1)
                    extra[key] = {"kernel": name, "kernel_fn": kernel_label(ist)["kernel_fn"],
                                  "kernel_ms_per_launch": round(ik, 4),
                                  "kernel_gcups": round(bcells / (ik * 1e-3) / 1e9, 3),
                                  "parity": ("ok" if isc == ref[:len(isc)] else "MISMATCH")
                                  if defaults and len(ref) >= 1024 else "unchecked"}
                finally:
                    sw.set_option("mode", args.mode if args.mode >= 0 else -1)
                    sw.set_option("f2pwg", -1)
                    sw.set_option("f3pwg", 1)
            if defaults and args.mode < 0:
                extra["affine_step"] = batch_affine_runs(sw, torch, gold, bsteps, params, bcells)

    value = cells_job * args.steps / t_max / 1e9
    if rank == 0:
        out = {
            "metric": "GCUPS (cell updates/s) for NxN affine-gap SW; bit-exact score vs CPU"
                      + ("; N>1: one C2-size pair per GPU (the batched pairs: batch_c4)"
                         if world > 1 and workload == "pair" else ""),
            "value": round(value, 3),
            "unit": "GCUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16x2 (packed, exact: scores < 2^16)" if st["mode"] == 3 else "int32",
            "data": "synthetic (uniform ACGT, mt19937_64 seeds as cudaSmithM.cu:200-212), resident in HBM",
            "config": dict(cfg, params=list(params), kernel_items=st["items"], blocks=st["blocks"],
                           boundary_bytes=st["boundary_bytes"], **kernel_label(st)),
            "kernel_ms_per_launch": round(avg_kern_ms, 4),
            "kernel_gcups": round(per_launch_cells / (avg_kern_ms * 1e-3) / 1e9, 3),
            "parity": parity,
            "host_api": host_api,
            "roofline": roofline((workload if args.slab_of <= 1 else "slab_part") + affine_key(st), per_launch_cells, avg_kern_ms,
                                 step_ns, cfg["N"], cfg["N"], bool(st["variant"] & 16),
                                 waves_per_simd=None if workload == "pair" else resident_waves_per_simd(st, torch)),
        }
        if rccl is not None:
            out["rccl_world"] = rccl
        if extra is not None:
            out["batch_c3" if world == 1 else "batch_c4"] = extra
        if slab_ranks is not None:
            out["slab_ranks"] = slab_ranks
        # the scaling series: `value` is the same per-GPU work at every N (one C2-size pair per
        # GPU), so value(N) / (N * value(1)) is the efficiency; the batched series is
        # batch_c4.value(N) against the N = 1 line's batch_c3.value (1024 pairs per GPU in both)
        if workload == "pair" and args.workload == "auto":
            out["scaling_note"] = ("value: one C2-size pair (N=%d) per GPU at every N; batched pairs: %s.value "
                                   "vs the N=1 line's batch_c3.value (1024 pairs N=8192 per GPU)"
                                   % (N, "batch_c3" if world == 1 else "batch_c4"))
        if workload != "batch" and affine is not None:
            out["affine_step"] = affine
        if workload != "batch" and c5 is not None:
            out["c5"] = c5
        if workload != "batch" and alpha is not None:
            out["byte_alphabets"] = alpha
        if world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(workload, cfg["N"], args.cpu_seconds, params)
            except Exception as e:   # the baseline leg must not kill the GPU number
                out["cpu_baseline"] = {"error": repr(e)}
        # last key of the line: every workload's step time, rate and parity in a few hundred bytes, so a
        # record that keeps only the tail of the output (the driver keeps 2000 characters) still holds them
        out["summary"] = headline_summary(out)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
