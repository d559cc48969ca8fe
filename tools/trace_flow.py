#!/usr/bin/env python3
"""Per-strip timeline of the flow kernels (mode 4, or 5 = flow2) on one long pair.

    python tools/trace_flow.py N C [W] [n_cols] [mode] [f2w]

Each strip records s_memrealtime (100 MHz) at start, when its first inflow
chunk arrived, and at the end, plus the number of failed progress polls.
Prints the inter-strip start lag (in-group LDS hops vs cross-group granule
hops), the run time per strip in ns/step and the poll counts."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import concurrentproject_amd as sw
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    ncol = int(sys.argv[4]) if len(sys.argv) > 4 else N
    mode = int(sys.argv[5]) if len(sys.argv) > 5 else 4
    f2w = int(sys.argv[6]) if len(sys.argv) > 6 else 0   # flow2 columns per lane (option f2w)
    torch.cuda.set_device(0)
    a, b = sw.gen_pair(N, N)
    a = a[:ncol]
    arena = torch.from_numpy(np.concatenate([a, b])).cuda()
    scores = torch.zeros(1, dtype=torch.int32, device="cuda")
    if mode != 5:
        strips = (ncol + 64 * W - 1) // (64 * W)
    elif f2w == 2:
        strips = 1 if ncol <= 128 else (ncol - 2 + 125) // 126
    else:
        strips = max(1, (ncol - 1 + 62) // 63)
    trace = torch.zeros(16 * strips, dtype=torch.int64, device="cuda")
    sw.set_option("mode", mode)
    sw.set_option("W", W)
    sw.set_option("C", C)
    sw.set_option("f2w", f2w)
    if os.environ.get("TRACE_PARAMS"):   # MATCH,MISMATCH,G_INIT,G_EXT
        sw.set_params(sw.Params(*(int(x) for x in os.environ["TRACE_PARAMS"].split(","))))
    for kv in os.environ.get("TRACE_OPTS", "").split():   # extra engine options k=v
        k, v = kv.split("=")
        sw.set_option(k, int(v))
    s = torch.cuda.current_stream()
    for it in range(3):
        if it == 2:
            sw.set_option("trace", trace.data_ptr())
        sw.set_option("orient", 1)   # a (ncol) across lanes, b (N rows) down
        sw.score_batch_device(arena.data_ptr(), [0], [ncol], [ncol], [N], scores.data_ptr(), flags=1, stream=s.cuda_stream)
        torch.cuda.synchronize()
    sw.set_option("trace", 0)
    sw.stream_status(s.cuda_stream)
    t = trace.cpu().numpy().reshape(strips, 16).astype(np.int64)
    if os.environ.get("TRACE_DUMP"):   # the raw per-strip records (s_memrealtime, 100 MHz)
        np.save(os.environ["TRACE_DUMP"], t)
    t0 = t[:, 0].min()
    start, first, end, spins = (t[:, 0] - t0) * 10, (t[:, 1] - t0) * 10, (t[:, 2] - t0) * 10, t[:, 3]   # ns
    lag = np.diff(first)
    ingroup = np.array([(k + 1) % 4 != 0 for k in range(strips - 1)], dtype=bool)
    run_ns = end - first
    steps = N + 64 * W - 1 if mode != 5 else N + 63
    out = {
        "N": N, "ncol": ncol, "C": C, "W": W, "score": int(scores.item()), "strips": strips,
        "total_ms": float(end.max()) / 1e6,
        "lag_ingroup_ns_median": float(np.median(lag[ingroup])) if lag.size else None,
        "lag_crossgroup_ns_median": float(np.median(lag[~ingroup])) if (~ingroup).any() else None,
        "lag_ingroup_ns_p90": float(np.percentile(lag[ingroup], 90)) if lag.size else None,
        "lag_crossgroup_ns_p90": float(np.percentile(lag[~ingroup], 90)) if (~ingroup).any() else None,
        "sum_lag_ms": float(lag.sum()) / 1e6 if lag.size else 0.0,
        "run_ns_per_step_median": float(np.median(run_ns)) / steps,
        "run_ns_per_step_last": float(run_ns[-1]) / steps,
        "run_ns_per_step_first": float(run_ns[0]) / steps,
        "spins_median": float(np.median(spins)), "spins_max": int(spins.max()),
        "start_spread_ms": float(start.max() - start.min()) / 1e6,
    }
    if t[:, 5].any():   # phase stamps (build/libswmi355_stamps.so): cycles per chunk
        nch = t[:, 7].astype(np.float64)
        for k, name in ((4, "pro"), (5, "run"), (6, "epi")):
            out["cyc_per_chunk_" + name] = float(np.median(t[:, k] / nch))
        out["cyc_per_chunk_strip0"] = [float(t[0, k] / nch[0]) for k in (4, 5, 6)]
        out["cyc_per_chunk_mid"] = [float(t[5, k] / nch[5]) for k in (4, 5, 6)]
        out["cyc_per_chunk_last"] = [float(t[-1, k] / nch[-1]) for k in (4, 5, 6)]
    if t[:, 12].any():   # timeline build: wall clock at chunks 1, 2, 3, 50, 1000
        tl = (t[:, 8:13] - t0) * 10
        d50 = np.diff(tl[:, 3]); d1000 = np.diff(tl[:, 4])
        med = lambda x: float(np.median(x)) if x.size else None
        out["steady_lag_ns_c50_median"] = med(d50)
        out["steady_lag_ns_c1000_median"] = med(d1000)
        out["steady_lag_ns_c1000_ingroup"] = med(d1000[ingroup])
        out["steady_lag_ns_c1000_crossgroup"] = med(d1000[~ingroup])
        out["chunk_ns_c50_c1000_median"] = float(np.median((tl[:, 4] - tl[:, 3]) / 950.0))
        out["chunk_ns_c1_c3_median"] = float(np.median((tl[:, 2] - tl[:, 0]) / 2.0))
        out["first_to_c1_ns_median"] = float(np.median(tl[:, 0] - first))
        for k in sorted({k for k in (0, 1, 2, 3, 4, 5, 500, strips - 1) if k < strips}):
            print("TL", k, [int(x) for x in tl[k]], int(first[k]))
    d_end = np.diff(end)
    out["lag_end_ns_median"] = float(np.median(d_end)) if d_end.size else None
    out["lag_end_ns_ingroup"] = float(np.median(d_end[ingroup])) if d_end.size else None
    out["lag_end_ns_crossgroup"] = float(np.median(d_end[~ingroup])) if (~ingroup).any() else None
    out["strip0_run_ns_per_step"] = float(end[0] - start[0]) / steps
    sl = spins[1:]
    xg = np.array([(k + 1) % 4 == 0 for k in range(strips - 1)], dtype=bool)
    out["slow_chunks_ingroup_mean"] = float(sl[~xg].mean()) if sl.size else None
    out["slow_chunks_crossgroup_mean"] = float(sl[xg].mean()) if xg.any() else None
    print(json.dumps(out))
    for k in sorted(set(range(0, min(9, strips))) | set(range(max(0, strips - 5), strips))):
        print(k, int(start[k]), int(first[k]), int(end[k]), int(spins[k]), round(run_ns[k] / steps, 2))
    # pace along the pipeline: ns per step of each strip's run (first inflow -> end)
    ks = list(range(0, strips, max(1, strips // 24)))
    print("pace", [(k, round(run_ns[k] / steps, 1)) for k in ks])
    print("end_lag_by_wave", [float(np.median(d_end[np.arange(d_end.size) % 4 == w])) for w in range(4)] if d_end.size else [])


if __name__ == "__main__":
    main()
