#!/usr/bin/env python3
"""Per-launch times over a long series of back-to-back launches (GPU): how the kernel time moves
from the first launch of a process to the steady state (clock ramp, first touch of the buffers).

    python tools/launch_series.py --work c3 --launches 40 [--params 2,-3,5,2] [--gap-ms 0]

--work c3: the C3 batch (1024 pairs of 8192, seeds 8192 + k) through sw_score_batch_device;
--work c2: the C2 pair.  One JSON line per launch, then a summary line."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", default="c3", choices=("c3", "c2"))
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--params", default="1,-1,1,1")
    ap.add_argument("--gap-ms", type=float, default=0.0, help="host sleep between launches")
    args = ap.parse_args()
    import torch
    import concurrentproject_amd as sw
    sw.set_params(sw.Params(*[int(x) for x in args.params.split(",")]))
    if args.work == "c3":
        N, P = 8192, 1024
        host = sw.gen_batch(8192, P, N)
        offa = [2 * N * k for k in range(P)]
        offb = [2 * N * k + N for k in range(P)]
        la = lb = [N] * P
    else:
        N, P = 65536, 1
        a, b = sw.gen_pair(N, N)
        host = np.concatenate([a, b])
        offa, offb, la, lb = [0], [N], [N], [N]
    arena = torch.from_numpy(host).cuda()
    scores = torch.zeros(P, dtype=torch.int32, device="cuda")
    s = torch.cuda.Stream()
    cells = sum(x * y for x, y in zip(la, lb))
    ms = []
    for i in range(args.launches):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        sw.score_batch_device(arena.data_ptr(), offa, la, offb, lb, scores.data_ptr(), flags=1, stream=s.cuda_stream)
        e1.record(s)
        s.synchronize()
        sw.stream_status(s.cuda_stream)
        t = e0.elapsed_time(e1)
        ms.append(t)
        print(json.dumps({"launch": i, "ms": round(t, 4)}), flush=True)
        if args.gap_ms > 0:
            time.sleep(args.gap_ms / 1e3)
    tail = sorted(ms[len(ms) // 2:])
    print(json.dumps({"work": args.work, "first": round(ms[0], 4), "second": round(ms[1], 4),
                      "mean_2_12": round(float(np.mean(ms[2:12])), 4),
                      "median_second_half": round(tail[len(tail) // 2], 4), "min": round(min(ms), 4),
                      "gcups_median_second_half": round(cells / tail[len(tail) // 2] / 1e6, 1),
                      "stats": sw.last_stats()}), flush=True)


if __name__ == "__main__":
    main()
