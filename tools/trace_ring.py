#!/usr/bin/env python3
"""Per-strip timeline of a ring-mode launch (flow3 ring kernels; tools only).

    python tools/trace_ring.py OUT.npz [f2w] [N]

Runs the C5 pair (seed 1048576, or N columns of it) once untraced and once with option trace
(sw_flow3.hip flow3_ring: per strip t_start, t_end in s_memrealtime ticks of 10 ns, failed polls,
HW_ID, XCC_ID) and saves the arrays with the launch's stats, for the schedule model
(tools/sim_ring.py) to be checked against."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import concurrentproject_amd as sw
    out = sys.argv[1]
    f2w = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    N = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    torch.cuda.set_device(0)
    a, b = sw.gen_pair(1048576, 1 << 20)
    a, b = a[:N], b[:N]
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    score = torch.zeros(1, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    sw.set_option("f2w", f2w)

    def launch():
        sw.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s.cuda_stream)

    launch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    launch()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    st = sw.last_stats()
    strips = 4 * st["items"]
    trace = torch.zeros(16 * strips, dtype=torch.int64, device="cuda")
    sw.set_option("trace", trace.data_ptr())
    try:
        launch()
        torch.cuda.synchronize()
    finally:
        sw.set_option("trace", 0)
    sw.stream_status(s.cuda_stream)
    t = trace.cpu().numpy().reshape(strips, 16)
    live = t[:, 0] > 0
    base = t[live, 0].min()
    np.savez_compressed(out, start=(t[:, 0] - base) * 10.0, end=(t[:, 2] - base) * 10.0, slow=t[:, 3],
                        hwid=t[:, 4], xcc=t[:, 5], live=live)
    info = {"ms_untraced": round(ms, 3), "score": int(score.item()), "stats": st,
            "span_ms_traced": float((t[live, 2].max() - base) * 1e-5)}
    print(json.dumps(info), flush=True)


if __name__ == "__main__":
    main()
