#!/usr/bin/env python3
"""C5: one pair of N = 1,048,576 (seed 1048576).  Scores it with the default
plan, with the transposed problem and with another strip width; all must agree
(size-independent parity properties while the CPU golden is pending)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import concurrentproject_amd as sw
    torch.cuda.set_device(0)
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    a, b = sw.gen_pair(N, N)
    host = np.concatenate([a, b])
    arena = torch.from_numpy(host).cuda()
    scores = torch.zeros(1, dtype=torch.int32, device="cuda")
    out = {"N": N, "runs": []}
    for label, opts, swap in (("default", {}, False), ("transposed", {}, True), ("W4", {"W": 4}, False),
                              ("default-again", {}, False)):
        for k in ("W", "C"):
            sw.set_option(k, opts.get(k, 0))
        offa, offb = ([N], [0]) if swap else ([0], [N])
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.time()
        e0.record(s)
        sw.score_batch_device(arena.data_ptr(), offa, [N], offb, [N], scores.data_ptr(), flags=1, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        sw.stream_status(s.cuda_stream)
        ms = e0.elapsed_time(e1)
        st = sw.last_stats()
        out["runs"].append({"run": label, "score": int(scores.item()), "ms": round(ms, 2),
                            "gcups": round(N * N / ms / 1e6, 1), "W": st["W"], "C": st["C"], "mode": st["mode"],
                            "boundary_GB": round(st["boundary_bytes"] / 1e9, 2), "wall_s": round(time.time() - t0, 2)})
        print(json.dumps(out["runs"][-1]), flush=True)
    assert len({r["score"] for r in out["runs"]}) == 1, "C5 runs disagree"
    print(json.dumps({"C5_score": out["runs"][0]["score"], "agree": True}))


if __name__ == "__main__":
    main()
