#!/usr/bin/env python3
"""Pin the batch goldens and the affine-gap goldens to the reference's own code.

TEST INFRASTRUCTURE (build container only: it needs oracle/_ref, compiled in place from
/root/reference by `make -C oracle ref refvar MA=2 MI=-3 GI=5 GE=2`).

  --c4        score all 8192 C4 pairs (seeds 8192+k, N = 8192; C3 is the first 1024) with
              the reference's LazySmith (lazySmith.cpp:15-69) on a thread pool (ctypes drops
              the GIL), check them against the committed scores, and record the provenance
              in configs.json C3 / C4 ("pinned_by").
  --affine    G_INIT != G_EXT goldens at config size, params (2, -3, 5, 2): the C2 pair
              (seed 65536, N = 65536) and the first 64 C3 pairs, each scored by the
              reference's LazySmith built with those constants (refvar, main.cpp:20-23
              substituted on a pipe, no edited source) AND by the oracle's restatement
              (swo_linear); written only when both agree, as configs.json C2_affine /
              C3_affine.
  --similar   the same at C2 size on oracle.similar_pair(7, 65536) (long alignments, long gaps),
              as configs.json C2_affine_similar.
  --c3similar  C3's shape with long E/F legs: oracle.similar_pair(8192 + k, 8192), k < --npairs,
              at (2, -3, 5, 2), by the reference's refvar LazySmith and swo_linear, as
              configs.json C3_affine_similar.
  --c5similar ENGINE  oracle.similar_pair(20, 2^20) at (2, -3, 5, 2) (the C5-size E/F-heavy pair),
              ENGINE "ref" or "wavefront" as for --c5affine; writes
              tests/golden/c5_affine_similar_<engine>.json; --merge-c5 also writes
              configs.json C5_affine_similar when the results present agree.
  --c5affine ENGINE   the C5 pair (seed 1048576, N = 2^20) at (2, -3, 5, 2): ENGINE "ref" (the
              reference's LazySmith refvar build, 1 thread, hours) or "wavefront" (the oracle's
              pthread restatement); writes tests/golden/c5_affine_<engine>.json; --merge-c5 then
              writes configs.json C5_affine when every result present agrees.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

AFF = oracle.Params(2, -3, 5, 2)
PATH = os.path.join(HERE, "configs.json")


def sha(a, b):
    h = hashlib.sha256()
    h.update(np.asarray(a, np.uint8).tobytes()); h.update(b"|"); h.update(np.asarray(b, np.uint8).tobytes())
    return h.hexdigest()


def ref_lazy(prm):
    L = oracle.ref_lib(prm)
    if L is None:
        raise SystemExit("oracle/_ref build missing for %s: make -C oracle ref refvar" % (prm,))
    return lambda a, b: oracle.ref_score(a, b, prm, which="lazy")


def pool_scores(fn, seeds, N, threads):
    def one(seed):
        a, b = oracle.gen_pair(seed, N)
        return fn(a, b)
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(one, seeds))


def pin_c4(threads: int) -> None:
    cfg = json.load(open(PATH))
    fn = ref_lazy(oracle.DEFAULT)
    t0 = time.time()
    sc = []
    for k0 in range(0, 8192, 512):
        sc += pool_scores(fn, range(8192 + k0, 8192 + k0 + 512), 8192, threads)
        print("C4 ref", k0 + 512, round(time.time() - t0, 1), "s", flush=True)
    dt = time.time() - t0
    assert sc == cfg["C4"]["scores"], "reference LazySmith disagrees with the committed C4 scores"
    assert sc[:1024] == cfg["C3"]["scores"]
    src = ("reference LazySmith (lazySmith.cpp:15-69) compiled from /root/reference, all %d pairs, "
           "%d threads, %.0f s (tests/golden/gen_pin.py --c4)")
    cfg["C4"]["pinned_by"] = [src % (8192, threads, dt), "oracle swo_linear (sw_oracle.c, lazySmith.cpp:15-42 restated)"]
    cfg["C3"]["pinned_by"] = [src % (1024, threads, dt) + ": the first 1024 of C4",
                              "oracle swo_linear (sw_oracle.c, lazySmith.cpp:15-42 restated)"]
    json.dump(cfg, open(PATH, "w"), indent=1)
    print("C4 pinned", dt)


def pin_affine(threads: int, npairs: int) -> None:
    cfg = json.load(open(PATH))
    fn = ref_lazy(AFF)
    t0 = time.time()
    a, b = oracle.gen_pair(65536, 65536)
    r = fn(a, b)
    t_ref = time.time() - t0
    o = oracle.score_linear(a, b, AFF)
    assert r == o, (r, o)
    cfg["C2_affine"] = {"seed": 65536, "N": 65536, "params": [AFF.match, AFF.mismatch, AFF.gap_init, AFF.gap_ext], "score": int(r), "sha256": sha(a, b),
                        "pinned_by": ["reference LazySmith built with (2,-3,5,2) (oracle/Makefile refvar) in %.0f s"
                                      % t_ref, "oracle swo_linear"]}
    print("C2_affine", r, round(t_ref, 1), flush=True)
    t0 = time.time()
    sc = pool_scores(fn, range(8192, 8192 + npairs), 8192, threads)
    t_ref = time.time() - t0
    so = pool_scores(lambda x, y: oracle.score_linear(x, y, AFF), range(8192, 8192 + npairs), 8192, threads)
    assert sc == so
    cfg["C3_affine"] = {"seed_base": 8192, "N": 8192, "npairs": npairs, "params": [AFF.match, AFF.mismatch, AFF.gap_init, AFF.gap_ext], "scores": sc,
                        "pinned_by": ["reference LazySmith built with (2,-3,5,2) (oracle/Makefile refvar), "
                                      "%d threads, %.0f s" % (threads, t_ref), "oracle swo_linear"]}
    print("C3_affine", sc[:8], round(t_ref, 1), flush=True)
    json.dump(cfg, open(PATH, "w"), indent=1)


def pin_similar() -> None:
    cfg = json.load(open(PATH))
    fn = ref_lazy(AFF)
    a, b = oracle.similar_pair(7, 65536)
    t0 = time.time()
    r = fn(a, b)
    t_ref = time.time() - t0
    o = oracle.score_linear(a, b, AFF)
    assert r == o, (r, o)
    cfg["C2_affine_similar"] = {"generator": "oracle.similar_pair(7, 65536)", "N": 65536,
                                "params": [AFF.match, AFF.mismatch, AFF.gap_init, AFF.gap_ext], "score": int(r),
                                "sha256": sha(a, b),
                                "pinned_by": ["reference LazySmith built with (2,-3,5,2) (oracle/Makefile refvar) "
                                              "in %.0f s" % t_ref, "oracle swo_linear"]}
    json.dump(cfg, open(PATH, "w"), indent=1)
    print("C2_affine_similar", r, round(t_ref, 1), flush=True)


def pin_c3_similar(threads: int, npairs: int) -> None:
    fn = ref_lazy(AFF)

    def one_ref(k):
        a, b = oracle.similar_pair(8192 + k, 8192)
        return fn(a, b)

    def one_oracle(k):
        a, b = oracle.similar_pair(8192 + k, 8192)
        return oracle.score_linear(a, b, AFF)

    t0 = time.time()
    with ThreadPoolExecutor(threads) as ex:
        sc = list(ex.map(one_ref, range(npairs)))
    t_ref = time.time() - t0
    with ThreadPoolExecutor(threads) as ex:
        so = list(ex.map(one_oracle, range(npairs)))
    assert sc == so, [k for k in range(npairs) if sc[k] != so[k]][:8]
    cfg = json.load(open(PATH))
    cfg["C3_affine_similar"] = {
        "generator": "oracle.similar_pair(8192 + k, 8192), k < npairs", "seed_base": 8192, "N": 8192,
        "npairs": npairs, "params": [AFF.match, AFF.mismatch, AFF.gap_init, AFF.gap_ext], "scores": sc,
        "pinned_by": ["reference LazySmith built with (2,-3,5,2) (oracle/Makefile refvar), "
                      "%d threads, %.0f s (tests/golden/gen_pin.py --c3similar)" % (threads, t_ref),
                      "oracle swo_linear"]}
    json.dump(cfg, open(PATH, "w"), indent=1)
    print("C3_affine_similar", sc[:8], min(sc), max(sc), round(t_ref, 1), flush=True)


C5_SIMILAR_SEED = 20


def c5_affine(engine: str, threads: int, similar: bool = False) -> None:
    if similar:
        a, b = oracle.similar_pair(C5_SIMILAR_SEED, 1 << 20)
    else:
        a, b = oracle.gen_pair(1048576, 1 << 20)
    t0 = time.time()
    if engine == "ref":
        s = ref_lazy(AFF)(a, b)
        src = "reference LazySmith built with (2,-3,5,2) (oracle/Makefile refvar), 1 thread"
    else:
        s = oracle.score_wavefront(a, b, AFF, threads=threads)
        src = "oracle swo_wavefront (sw_oracle.c, main.cpp:54-66 restated), %d threads" % threads
    out = {"seed": 1048576, "N": 1 << 20, "params": [AFF.match, AFF.mismatch, AFF.gap_init, AFF.gap_ext],
           "score": int(s), "seconds": round(time.time() - t0, 1), "sha256": sha(a, b), "source": src}
    name = "c5_affine_%s.json" % engine
    if similar:
        del out["seed"]
        out["generator"] = "oracle.similar_pair(%d, 2^20)" % C5_SIMILAR_SEED
        name = "c5_affine_similar_%s.json" % engine
    json.dump(out, open(os.path.join(HERE, name), "w"), indent=1)
    print(json.dumps(out), flush=True)


def merge_c5_similar() -> None:
    res = [json.load(open(os.path.join(HERE, "c5_affine_similar_%s.json" % e))) for e in ("ref", "wavefront")
           if os.path.exists(os.path.join(HERE, "c5_affine_similar_%s.json" % e))]
    if not res:
        return
    assert len({r["score"] for r in res}) == 1 and len({r["sha256"] for r in res}) == 1
    cfg = json.load(open(PATH))
    cfg["C5_affine_similar"] = {"generator": res[0]["generator"], "N": 1 << 20, "params": res[0]["params"],
                                "score": res[0]["score"], "sha256": res[0]["sha256"],
                                "pinned_by": [r["source"] + " in %.0f s" % r["seconds"] for r in res]}
    json.dump(cfg, open(PATH, "w"), indent=1)
    print("C5_affine_similar", cfg["C5_affine_similar"])


def merge_c5() -> None:
    res = [json.load(open(os.path.join(HERE, "c5_affine_%s.json" % e))) for e in ("ref", "wavefront")
           if os.path.exists(os.path.join(HERE, "c5_affine_%s.json" % e))]
    assert res and len({r["score"] for r in res}) == 1 and len({r["sha256"] for r in res}) == 1
    cfg = json.load(open(PATH))
    cfg["C5_affine"] = {"seed": 1048576, "N": 1 << 20, "params": res[0]["params"], "score": res[0]["score"],
                        "sha256": res[0]["sha256"],
                        "pinned_by": [r["source"] + " in %.0f s" % r["seconds"] for r in res]}
    json.dump(cfg, open(PATH, "w"), indent=1)
    print("C5_affine", cfg["C5_affine"])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--c4", action="store_true")
    ap.add_argument("--affine", action="store_true")
    ap.add_argument("--threads", type=int, default=7)
    ap.add_argument("--npairs", type=int, default=64)
    ap.add_argument("--similar", action="store_true")
    ap.add_argument("--c5affine", choices=["ref", "wavefront"])
    ap.add_argument("--merge-c5", action="store_true")
    ap.add_argument("--c3similar", action="store_true")
    ap.add_argument("--c5similar", choices=["ref", "wavefront"])
    args = ap.parse_args()
    if args.similar:
        pin_similar()
    if args.c5affine:
        c5_affine(args.c5affine, args.threads)
    if args.c5similar:
        c5_affine(args.c5similar, args.threads, similar=True)
    if args.merge_c5:
        merge_c5()
        merge_c5_similar()
    if args.c3similar:
        pin_c3_similar(args.threads, args.npairs)
    if args.affine:
        pin_affine(args.threads, args.npairs)
    if args.c4:
        pin_c4(args.threads)
