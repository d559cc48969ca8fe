#!/usr/bin/env python3
"""Where the duo LDS kernel's waves run and when they finish (GPU): C3 with the trace
option; per wave HW_ID (SIMD, CU, SH, SE), XCC_ID, begin and end (s_memrealtime, 100 MHz).
Prints how strip roles map to SIMDs on the CUs that hold two workgroups, and the per-SIMD
idle time at the start and end of the launch.

    python tools/probe_duo_simd.py [duo_tab [duo_prio]]
"""
import collections
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import concurrentproject_amd as sw
    rev = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    N, P = 8192, 1024
    host = sw.gen_batch(8192, P, N)
    arena = torch.from_numpy(host).cuda()
    scores = torch.zeros(P, dtype=torch.int32, device="cuda")
    offs_a = [2 * N * k for k in range(P)]
    offs_b = [2 * N * k + N for k in range(P)]
    sw.set_option("duo_tab", rev)
    if len(sys.argv) > 2:
        sw.set_option("duo_prio", int(sys.argv[2]))
    s = torch.cuda.current_stream()
    trace = None
    for it in range(3):
        if it == 2:
            st = sw.last_stats()
            trace = torch.zeros(16 * st["blocks"], dtype=torch.int64, device="cuda")
            sw.set_option("trace", trace.data_ptr())
        sw.score_batch_device(arena.data_ptr(), offs_a, [N] * P, offs_b, [N] * P, scores.data_ptr(), flags=1,
                              stream=s.cuda_stream)
        torch.cuda.synchronize()
    sw.set_option("trace", 0)
    sw.stream_status(s.cuda_stream)
    t = trace.cpu().numpy().reshape(-1, 4).astype(np.int64)
    hw = t[:, 0] & 0xFFFFFFFF
    role = (t[:, 0] >> 40) & 0xF
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = t[:, 1] & 0xF
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    t0 = t[:, 2].min()
    beg, end = (t[:, 2] - t0) / 100.0, (t[:, 3] - t0) / 100.0   # us
    print("waves", len(t), "CUs", len(set(key)), "kernel span us %.1f" % (end.max() - beg.min()))
    print("begin us: min %.1f p25 %.1f median %.1f p75 %.1f max %.1f" % tuple(np.percentile(beg, [0, 25, 50, 75, 100])))
    print("end us:   min %.1f p25 %.1f median %.1f p75 %.1f max %.1f" % tuple(np.percentile(end, [0, 25, 50, 75, 100])))
    late = beg > 0.25 * end.max()
    print("waves beginning after a quarter of the span: %d of %d" % (int(late.sum()), len(t)))
    # workgroups whose waves overlap in time on one CU
    by_cu = collections.defaultdict(list)
    for i in range(0, len(t), 4):
        by_cu[int(key[i])].append((float(beg[i:i + 4].min()), float(end[i:i + 4].max())))
    conc = sum(1 for v in by_cu.values() for a in v for b in v if a < b and a[0] < b[1] and b[0] < a[1])
    print("CUs with 2+ workgroups: %d; overlapping workgroup pairs: %d" % (sum(len(v) > 1 for v in by_cu.values()), conc))
    m = collections.Counter((int(r), int(sm)) for r, sm in zip(role, simd))
    print("role -> SIMD counts:", dict(sorted(m.items())))
    per = collections.defaultdict(list)
    for i in range(len(t)):
        per[(int(key[i]), int(simd[i]))].append((float(beg[i]), float(end[i]), int(role[i])))
    idle_start, idle_end, pairs = [], [], collections.Counter()
    span_end = end.max()
    for k, v in per.items():
        pairs[tuple(sorted(r for _, _, r in v))] += 1
        idle_end.append(span_end - max(e for _, e, _ in v))
    print("roles sharing a SIMD:", dict(pairs.most_common(8)))
    ends = sorted(end)
    print("end us: min %.1f median %.1f max %.1f; SIMD idle at the end: median %.1f us" %
          (ends[0], ends[len(ends) // 2], ends[-1], float(np.median(idle_end))))
    wg_end = [sorted(e for _, e in v) for v in by_cu.values() if len(v) == 2]
    if wg_end:
        print("workgroup end per CU: first median %.1f us, second median %.1f us" %
              (float(np.median([w[0] for w in wg_end])), float(np.median([w[1] for w in wg_end]))))
    for r in range(4):
        sel = role == r
        print("role %d: end median %.1f us" % (r, float(np.median(end[sel]))))


if __name__ == "__main__":
    main()
