"""Diagnostic: flow2 ring mode at several workgroups per CU on one long pair, with the
strip trace on; on a time-out, which strips stalled first.

    python tools/probe_ring.py N WGS [timeout_s] [blocks]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import concurrentproject_amd as sw

torch.cuda.set_device(0)
N = int(sys.argv[1])
W = int(sys.argv[2])
sw.set_option("timeout", int(sys.argv[3]) if len(sys.argv) > 3 else 5)
if len(sys.argv) > 4:
    sw.set_option("blocks", int(sys.argv[4]))
a, b = sw.gen_pair(N, N)
arena = torch.from_numpy(np.concatenate([a, b])).cuda()
score = torch.zeros(1, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
strips = (N - 1 + 62) // 63
trace = torch.zeros(16 * strips, dtype=torch.int64, device="cuda")
sw.set_option("ring", 1)
sw.set_option("f2_wgs", W)
sw.set_option("trace", trace.data_ptr())
t = time.time()
err = None
try:
    sw.score_batch_device(arena.data_ptr(), [0], [N], [N], [N], score.data_ptr(), flags=1, stream=s)
    sw.stream_status(s)
except Exception as e:
    err = e
sw.set_option("trace", 0)
torch.cuda.synchronize()
st = sw.last_stats()
print("N", N, "wgs", W, "blocks", st["blocks"], "items", st["items"], "variant", st["variant"], "score", score.item(),
      "s %.2f" % (time.time() - t), "error", err, flush=True)
tr = trace.cpu().numpy().reshape(strips, 16).astype(np.int64)
t0 = tr[:, 0][tr[:, 0] > 0].min()
start = (tr[:, 0] - t0) / 1e5   # ms
end = (tr[:, 2] - t0) / 1e5
dur = end - start
groups = strips // 4
never = np.where(tr[:, 0] == 0)[0]
print("strips never traced:", len(never), "first groups", sorted(set((never // 4).tolist()))[:16])
g0 = start[0:4 * min(groups, st["blocks"]):4]
late = np.where(g0 > 0.5)[0]
print("round-0 groups starting after 0.5 ms:", len(late), late[:16].tolist(), np.round(g0[late[:16]], 2).tolist())
if err is not None:
    slow = np.where(dur > 0.5 * float(sys.argv[3] if len(sys.argv) > 3 else 5) * 1e3)[0]
    print("strips over half the time-out:", len(slow), "first", slow[:12].tolist())
    if len(slow):
        first = slow[np.argsort(start[slow])][:12]
        for k in first:
            g = k // 4
            print(" strip", k, "group", g, "block", g % st["blocks"], "round", g // st["blocks"],
                  "start %.2f end %.2f" % (start[k], end[k]), "fail_in", tr[k, 13], "fail_bp", tr[k, 14])
    fi = np.where(((tr[:, 13] >= 0) | (tr[:, 14] >= 0)) & (tr[:, 0] > 0))[0]
    print("strips with a recorded failure:", len(fi))
    for k in fi[:16]:
        print(" strip", k, "group", k // 4, "fail_in", tr[k, 13], "fail_bp", tr[k, 14],
              "start %.2f end %.2f" % (start[k], end[k]))
    lo = max(0, fi[0] // 4 - 2) * 4 if len(fi) else 0
    for k in range(lo, lo + 20):
        print(" ctx strip", k, "start %.2f end %.2f dur %.2f" % (start[k], end[k], dur[k]), "fail_in", tr[k, 13],
              "fail_bp", tr[k, 14])
else:
    print("max strip duration ms %.2f" % dur.max())
