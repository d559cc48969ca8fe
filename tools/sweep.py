#!/usr/bin/env python3
"""Performance sweep of the score kernel (GPU).  Prints one JSON line per case.

    python tools/sweep.py [--cases spec,...]

Case spec: kind:n:m[:W[:C[:npairs[:mode]]]]   kind = pair | batch; mode -1 auto, 0 strip, 1 pairwg, 2 chain
  pair:64:65536:1:16      one strip of 64 columns x 65536 rows (per-step cost, no hand-offs)
  pair:65536:65536:1:16   the C2 config
  batch:8192:8192:8:64:1024  the C3 config
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = ("pair:64:65536:1:16,pair:64:65536:1:32,pair:512:65536:8:64,"
           "pair:65536:65536:1:16,pair:65536:65536:1:32,pair:65536:65536:1:16:1:0,pair:65536:65536:2:32,"
           "pair:65536:65536:4:64,pair:1024:65536:1:16,pair:1024:65536:1:32,"
           "batch:8192:8192:8:64:1024,batch:8192:8192:8:64:1024:0,batch:8192:8192:4:64:1024,"
           "batch:8192:8192:2:32:1024,batch:512:65536:8:64:1024")


def run_case(sw, torch, spec, reps):
    f = spec.split(":")
    kind, n, m = f[0], int(f[1]), int(f[2])
    W = int(f[3]) if len(f) > 3 else 0
    C = int(f[4]) if len(f) > 4 else 0
    P = int(f[5]) if len(f) > 5 else 1
    mode = int(f[6]) if len(f) > 6 else -1
    sw.set_option("mode", mode)
    sw.set_option("W", W)
    sw.set_option("C", C)
    sw.set_option("orient", 1)      # seq1 (length n) across the lanes, as written in the spec
    if kind == "pair":
        a, b = sw.gen_pair(65536, max(n, m))
        host = np.concatenate([a[:n], b[:m]])
        offa, offb, la, lb = [0], [n], [n], [m]
    else:
        host = sw.gen_batch(8192, P, max(n, m))
        L = max(n, m)
        offa = [2 * L * k for k in range(P)]
        offb = [2 * L * k + L for k in range(P)]
        la, lb = [n] * P, [m] * P
    arena = torch.from_numpy(host).cuda()
    scores = torch.zeros(len(la), dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()

    def go():
        sw.score_batch_device(arena.data_ptr(), offa, la, offb, lb, scores.data_ptr(), flags=1,
                              stream=s.cuda_stream)
    go(); go()
    sw.stream_status(s.cuda_stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(s); go(); e1.record(s)
    torch.cuda.synchronize()
    sw.stream_status(s.cuda_stream)
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    st = sw.last_stats()
    cells = sum(x * y for x, y in zip(la, lb))
    med = ms[len(ms) // 2]
    steps = m + 64 * st["W"] - 1
    return {"case": spec, "mode": st["mode"], "W": st["W"], "C": st["C"], "items": st["items"], "blocks": st["blocks"],
            "ms_med": round(med, 4), "ms_min": round(ms[0], 4), "gcups": round(cells / med / 1e6, 2),
            "ns_per_strip_step": round(med * 1e6 / steps, 2) if n <= 64 * st["W"] else None,
            "score0": int(scores[0].item()), "scores_sum": int(scores.sum().item()),
            "variant": st["variant"], "waves_per_cu": st["waves_per_cu"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default=DEFAULT)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--opt", action="append", default=[], help="engine option k=v (sw_set_option), repeatable")
    args = ap.parse_args()
    import torch
    import concurrentproject_amd as sw
    torch.cuda.set_device(0)
    for kv in args.opt:
        k, v = kv.split("=")
        sw.set_option(k, int(v))
    for spec in args.cases.split(","):
        t0 = time.time()
        try:
            r = run_case(sw, torch, spec, args.reps)
        except Exception as e:
            r = {"case": spec, "error": repr(e)}
        r["wall_s"] = round(time.time() - t0, 2)
        print(json.dumps(r), flush=True)
    for k in ("W", "C", "orient"):
        sw.set_option(k, 0)
    sw.set_option("mode", -1)


if __name__ == "__main__":
    main()
